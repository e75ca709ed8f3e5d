#!/bin/bash
# Round 4: the tests that failed in r04_full, then the B&B host profile after the batched flows / pinned submit
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_fix}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_solvers.py tests/test_gpu_bnb_parity.py tests/test_gpu_fac.py tests/test_gpu_stream.py tests/test_gpu_params.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|XFAIL|ERROR|passed|failed|^testpy|^payload " "$O/pytest.log" | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"
[ $rc -eq 0 ] || exit $rc
for kn in '{}' '{"leaf_warm_incumbent": true}'; do
  MODES=two KNOBS="$kn" timeout -k 10 200 python -u tools/bnb_fac_probe.py 256x128:20 512x256:20 > "$O/bnb_$(echo $kn | tr -dc a-z).log" 2>&1
  rc=$?; echo "bnb [$kn] rc=$rc"; grep "two" "$O/bnb_$(echo $kn | tr -dc a-z).log"
  [ $rc -eq 0 ] || exit $rc
done
