#!/bin/bash
# round 2, call AY: node LPs in flight per GPU (32 / 48 / 64; same 768 nodes) on seeds 0 and 1
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ay; mkdir -p $O
for bs in "32 24" "48 16" "64 12"; do set -- $bs; for s in 0 1; do
  timeout -k 10 300 python -u bench.py --batch $1 --steps $2 --seed $s --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/b_$1_$s.json 2> $O/b_$1_$s.log
  rc=$?; [ $rc -eq 0 ] || { echo "batch $1 s $s rc=$rc"; tail -3 $O/b_$1_$s.log; exit $rc; }
  python -c "import json;d=json.load(open('$O/b_$1_$s.json'));l=d['lp'];print('batch $1 seed $s', round(d['value'],1), round(d['ms_per_step'],1), l['certified'], l['completed'], round(l['mean_iters'],1), round(l['slot_utilisation_rank0'],3), round(d['roofline']['frac'],3), round(d['roofline']['avg_launch_ms'],3))"
done; done
