#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -30
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
timeout -k 10 300 python -u bench.py --cpu-budget 0 > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['lp'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3)); print(d['bnb'])"
