#!/bin/bash
# Round 4: testpy's LIMIT leaves vs HiGHS; the facility MU root's stall under primal-weight / restart knobs;
# the B&B host profile
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_diag}; mkdir -p "$O"
timeout -k 10 120 python -u tools/leaf_limit_probe.py testpy > "$O/leaf_testpy.log" 2>&1
rc=$?; echo "leaf rc=$rc"; grep -v "amdgpu\|Initializ" "$O/leaf_testpy.log" | tail -12
[ $rc -eq 0 ] || exit $rc
for knob in "" "NEP_OMEGA_SMOOTH=0.2" "NEP_OMEGA_SMOOTH=0.8" "NEP_RESTART=0.2,0.8,0.36" "NEP_RESTART=0.1,0.9,0.5"; do
  env $knob CHUNK=400000 CHUNKS=1 timeout -k 10 120 python -u tools/fac_conv_probe.py 32x16:MinUtilization > "$O/conv_$knob.log" 2>&1
  rc=$?; echo "conv [$knob] rc=$rc"; grep "LP" "$O/conv_$knob.log" | tail -5
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"; exit $rc
