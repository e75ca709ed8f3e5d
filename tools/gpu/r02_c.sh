#!/bin/bash
# round 2, call C: at-scale parity tests + params test, then a default bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_params.py tests/test_gpu_scale.py -v --timeout 300 --timeout-method thread -s > $O/pytest_scale.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_scale.log | tail -30
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
timeout -k 10 300 python -u bench.py --cpu-budget 0 > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; cut -c1-600 $O/bench.json
exit $rc
