#!/bin/bash
# round 2, call BA: pipelining policy — skip the pipelined block when more than K slots just finished (K = inf / 0 / 2)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ba; mkdir -p $O
for K in 1000000 0 2; do for s in 0 1; do
  NEP_PIPELINE_MAX_DONE=$K timeout -k 10 300 python -u bench.py --seed $s --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/b_${K}_$s.json 2> $O/b_${K}_$s.log
  rc=$?; [ $rc -eq 0 ] || { echo "K $K s $s rc=$rc"; tail -3 $O/b_${K}_$s.log; exit $rc; }
  python -c "import json;d=json.load(open('$O/b_${K}_$s.json'));l=d['lp'];print('K $K seed $s', round(d['value'],1), round(d['ms_per_step'],1), l['certified'], round(l['mean_iters'],1), round(l['slot_utilisation_rank0'],3))"
done; done
