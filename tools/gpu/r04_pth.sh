#!/bin/bash
# Round 4: threaded node presolve (NEP_PRESOLVE_THREADS) — product B&B host profile A/B + the B&B GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_pth}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_bnb.py tests/test_gpu_bnb_parity.py tests/test_gpu_bnb_dist.py -x -v --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 256x128:20 64x32:10 > "$O/profile_t8.log" 2>&1
rc=$?; echo "t8 rc=$rc"; grep "^==" "$O/profile_t8.log"; [ $rc -eq 0 ] || exit $rc
NEP_PRESOLVE_THREADS=1 timeout -k 10 150 python -u tools/bnb_profile.py 256x128:20 > "$O/profile_t1.log" 2>&1
rc=$?; echo "t1 rc=$rc"; grep "^==" "$O/profile_t1.log"; exit $rc
