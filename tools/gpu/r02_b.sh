#!/bin/bash
# round 2, call B: tail probe (fp32 anchor, nt streams) with per-family residuals
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 400 python -u tools/tail_probe.py --probe-nodes 192 > $O/tail_probe.log 2>&1
rc=$?; echo "tail rc=$rc"; head -5 $O/tail_probe.log | cut -c1-300
exit $rc
