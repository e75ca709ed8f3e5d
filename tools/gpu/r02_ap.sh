#!/bin/bash
# round 2, call AP: diagnostics of the bench children that end at the node-LP limit (seeds 0 and 1)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ap; mkdir -p $O
for s in 0 1; do
timeout -k 10 300 python -u tools/tail_probe.py --seed $s --probe-nodes 128 --root-max-iters 1000000 > $O/tail_s$s.log 2>&1
rc=$?; echo "tail s$s rc=$rc"; grep -v "amdgpu\|Initializ" $O/tail_s$s.log | cut -c1-260 | tail -40; [ $rc -eq 0 ] || exit $rc
done
