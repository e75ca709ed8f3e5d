#!/bin/bash
# Round 4: greedy incumbents + high-priority aux stream: B&B at 256x128 / 512x256 (20 s), host profile, the
# GPU tests touched this session
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_heur}; mkdir -p "$O"
export TMPDIR=/tmp
MODES=two timeout -k 10 200 python -u tools/bnb_fac_probe.py 256x128:20 512x256:20 > "$O/bnb.log" 2>&1
rc=$?; echo "bnb rc=$rc"; grep -v "amdgpu\|Initializ" "$O/bnb.log" | grep "two\|incumbent" | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_bnb.py tests/test_gpu_bnb_parity.py tests/test_gpu_fac.py tests/test_gpu_bnb_dist.py tests/test_gpu_solvers.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|ERROR|passed|failed" "$O/pytest.log" | tail -20; exit $rc
