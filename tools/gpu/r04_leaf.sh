#!/bin/bash
# Round 4: primal leaves from the facility relaxation (tools/leaf_probe.py)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_leaf}; mkdir -p "$O"; shift
timeout -k 10 ${SECS:-600} python -u tools/leaf_probe.py "$@" > "$O/leaf.log" 2>&1
rc=$?; echo "rc=$rc"; grep -v "amdgpu\|Initializ" "$O/leaf.log" | tail -40; exit $rc
