#!/bin/bash
# Round 4: facility LPs that hit the iteration limit (tools/fac_conv_probe.py), then the B&B probe with the
# capacity-greedy primal heuristic
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_conv}; mkdir -p "$O"
timeout -k 10 300 python -u tools/fac_conv_probe.py 32x16:MinUtilization 64x32:MinDelayAndUtilization > "$O/conv.log" 2>&1
rc=$?; echo "conv rc=$rc"; grep -v "amdgpu\|Initializ" "$O/conv.log" | tail -40
[ $rc -eq 0 ] || exit $rc
MODES=two timeout -k 10 300 python -u tools/bnb_fac_probe.py 64x32:20 256x128:40 512x256:60 > "$O/bnbfac.log" 2>&1
rc=$?; echo "bnbfac rc=$rc"; grep -v "amdgpu\|Initializ\|incumbent" "$O/bnbfac.log" | tail -30; exit $rc
