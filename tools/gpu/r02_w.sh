#!/bin/bash
# round 2, call W: why the CPU-row repair stops certification: tail probe on 64 bench children
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 300 python -u tools/tail_probe.py --probe-nodes 64 > $O/tail.log 2>&1
rc=$?; grep -v "amdgpu\|Initializ" $O/tail.log | cut -c1-320 | head -40; exit $rc
