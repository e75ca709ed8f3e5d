#!/bin/bash
# Round 4: the whole -m gpu suite, smoke(), the B&B host profile and the 64x32 step-2 certificate probe
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_suite}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rA --durations=25 --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest_gpu.log" | grep -v "PASSED" | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"; [ $rc -eq 0 ] || exit $rc
ITERS=100000 timeout -k 10 200 python -u tools/step2_cert_probe.py scale:syn64x32_MDU_s2delete 0 0 > "$O/s2delete.log" 2>&1
rc=$?; echo "s2delete rc=$rc"; grep -v "amdgpu\|Initializ" "$O/s2delete.log" | tail -14; exit $rc
