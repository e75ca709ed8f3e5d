#!/bin/bash
# round 2, call AZ: the full GPU suite at the final head
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02az; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -20; exit $rc
