#!/bin/bash
# round 2, call AV: node-LP certificate interval (check_every 8 / 12 / 16 / 24) on seeds 0 and 1
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02av; mkdir -p $O
for ce in 8 12 16 24; do for s in 0 1; do
  timeout -k 10 300 python -u bench.py --seed $s --check-every $ce --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/b_${ce}_$s.json 2> $O/b_${ce}_$s.log
  rc=$?; [ $rc -eq 0 ] || { echo "ce $ce s $s rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('$O/b_${ce}_$s.json'));l=d['lp'];print('ce $ce seed $s', round(d['value'],1), round(d['ms_per_step'],1), l['certified'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(l['slot_utilisation_rank0'],3))"
done; done
