#!/bin/bash
# Round 4: two-model B&B (facility relaxation bounds) vs the single-model search (tools/bnb_fac_probe.py)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_bnbfac}; mkdir -p "$O"; shift
timeout -k 10 ${SECS:-700} python -u tools/bnb_fac_probe.py "$@" > "$O/bnbfac.log" 2>&1
rc=$?; echo "rc=$rc"; grep -v "amdgpu\|Initializ\|incumbent" "$O/bnbfac.log" | tail -30; exit $rc
