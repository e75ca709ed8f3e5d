#!/bin/bash
# round 2, call AX: B&B returns the certified leaf's routing even when the incumbent polish re-solve fails;
# B&B, solver-flow and request GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ax; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bnb.py tests/test_gpu_solvers.py tests/test_gpu_request.py -v --timeout 300 --timeout-method thread -rf -s > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|polished" $O/pytest.log | cut -c1-300 | tail -12; exit $rc
