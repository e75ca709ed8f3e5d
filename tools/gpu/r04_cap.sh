#!/bin/bash
# Round 4: the facility relaxation with capacity rows scaled by n: GPU parity test, root/children probe,
# two-model B&B at BASELINE configs 2-4
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_cap}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fac.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest_fac.log" 2>&1
rc=$?; echo "pytest_fac rc=$rc"; grep "LP \|passed\|failed\|Error" "$O/pytest_fac.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/fac_probe.py 64x32 256x128 512x256 > "$O/fac_probe.log" 2>&1
rc=$?; echo "fac_probe rc=$rc"; tail -12 "$O/fac_probe.log"
[ $rc -eq 0 ] || exit $rc
MODES=two timeout -k 10 300 python -u tools/bnb_fac_probe.py 64x32:20 256x128:40 512x256:60 > "$O/bnbfac.log" 2>&1
rc=$?; echo "bnbfac rc=$rc"; grep -v "amdgpu\|Initializ\|incumbent" "$O/bnbfac.log" | tail -30; exit $rc
