#!/bin/bash
# round 2, call T: step-2 certificate with the disruption block kept exact (dblock_pass + G(lambda));
# the LP parity suites, uncertified step-2 LPs counted
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py -v -s --timeout 300 --timeout-method thread > $O/pytest_lp.log 2>&1
rc=$?; grep -c "UNCERTIFIED" $O/pytest_lp.log; grep -E "UNCERTIFIED|FAILED|passed|failed" $O/pytest_lp.log | cut -c1-250 | tail -30; exit $rc
