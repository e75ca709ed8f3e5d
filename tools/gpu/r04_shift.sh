#!/bin/bash
# Round 4: the certificate's loaded-row shift on the step-2 XFAIL LPs (test_gpu_lp / test_gpu_scale), then the
# B&B with greedy incumbents at 256x128 / 512x256
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_shift}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py -m gpu -v -s -rA --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest.log" | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
MODES=two timeout -k 10 200 python -u tools/bnb_fac_probe.py 256x128:20 512x256:20 > "$O/bnb.log" 2>&1
rc=$?; echo "bnb rc=$rc"; grep -v "amdgpu\|Initializ" "$O/bnb.log" | grep "two\|incumbent" | tail -14; exit $rc
