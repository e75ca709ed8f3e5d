#!/bin/bash
# Round 4: cold-root restart / primal-weight settings (tools/root_probe.py)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_root}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/root_probe.py base \
  "nec8:NEP_RESTART=0.2,0.8,0.36" "nec95:NEP_RESTART=0.2,0.95,0.36" "suf1:NEP_RESTART=0.1,0.9,0.36" \
  "suf3:NEP_RESTART=0.3,0.9,0.36" "art2:NEP_RESTART=0.2,0.9,0.2" "art5:NEP_RESTART=0.2,0.9,0.5" \
  "sm3:NEP_OMEGA_SMOOTH=0.3" "sm7:NEP_OMEGA_SMOOTH=0.7" "sm0:NEP_OMEGA_SMOOTH=0" > "$O/root.log" 2>&1
rc=$?; echo "root rc=$rc"; cat "$O/root.log" | grep -v Warn; exit $rc
