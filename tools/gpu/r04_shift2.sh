#!/bin/bash
# Round 4: step-2 repair within the D-row box + shifts aimed there (test_gpu_lp / test_gpu_scale), then the
# capacity greedy at the facility roots
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_shift2}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_solvers.py -m gpu -v -s -rA --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest.log" | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/greedy_probe.py 256x128 512x256 > "$O/greedy.log" 2>&1
rc=$?; echo "greedy rc=$rc"; grep -v "amdgpu\|Initializ" "$O/greedy.log" | tail -12; exit $rc
