#!/bin/bash
# round 2, call BC: polishing entry residual / budget (NEP_POLISH="res,budget") on seeds 0 and 1
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02bc; mkdir -p $O
for P in 1e-3,512 1e-2,512 1e-3,1024 1e-2,1024; do for s in 0 1; do
  NEP_POLISH=$P timeout -k 10 300 python -u bench.py --seed $s --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/b_${P}_$s.json 2> $O/b_${P}_$s.log
  rc=$?; [ $rc -eq 0 ] || { echo "P $P s $s rc=$rc"; tail -3 $O/b_${P}_$s.log; exit $rc; }
  python -c "import json;d=json.load(open('$O/b_${P}_$s.json'));l=d['lp'];print('P $P seed $s', round(d['value'],1), round(d['ms_per_step'],1), l['certified'], round(l['mean_iters'],1), l['iters_p50_p90_max'])"
done; done
