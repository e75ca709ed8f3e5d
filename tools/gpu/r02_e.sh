#!/bin/bash
# round 2, call E: repaired certificate with fp64 certificate sums: LP parity tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_stream.py tests/test_gpu_params.py -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -40
exit $rc
