#!/bin/bash
# round 2, call AJ: sensitivity of the warm children to primal-weight handling (seeds 0, 1)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02aj; mkdir -p $O
run() {
  local v=$1; shift
  timeout -k 10 240 env "$@" python -u bench.py --steps 4 --cpu-budget 0 --bnb-seconds 0 --root-gap-tol 0 --root-max-iters 1000000 --seed $SEED > $O/b_$v.json 2> $O/b_$v.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -2 $O/b_$v.log; return 0; }
  python -c "import json;d=json.load(open('$O/b_$v.json'));l=d['lp'];print('$v', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], l['root_iters'], round(d['ms_per_step'],1))"
}
for SEED in 0 1; do
run s${SEED}_base X=1
run s${SEED}_cap4 NEP_WARM_OMEGA_CAP=4
run s${SEED}_cap2 NEP_WARM_OMEGA_CAP=2
run s${SEED}_sm0 NEP_OMEGA_SMOOTH=0.0
done
