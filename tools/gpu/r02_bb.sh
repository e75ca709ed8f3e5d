#!/bin/bash
# round 2, call BB: the node LPs still uncertified at the limit with polishing (seeds 0 and 1, 256 nodes each)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02bb; mkdir -p $O
for s in 0 1; do
timeout -k 10 300 python -u tools/tail_probe.py --seed $s --probe-nodes 256 --root-max-iters 1000000 > $O/tail_s$s.log 2>&1
rc=$?; echo "tail s$s rc=$rc"; grep -v "amdgpu\|Initializ" $O/tail_s$s.log | cut -c1-250 | grep -v "^re-solve\|fix \[" | tail -14; [ $rc -eq 0 ] || exit $rc
done
