#!/bin/bash
# round 2, call AS: the request boundary (core.request) on the GPU, in process and in a forked child
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_request.py -v --timeout 500 --timeout-method thread -rf > $O/pytest_request.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" $O/pytest_request.log | tail -20; exit $rc
