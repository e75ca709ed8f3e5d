#!/bin/bash
# round 2, call M: restart / primal-weight parameter sweep on the bench workload
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02m; mkdir -p $O
run() {  # name, env assignments..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 12 --cpu-budget 0 --bnb-seconds 0 ${BARGS:-} > $O/b_$name.json 2> $O/b_$name.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 $O/b_$name.log; return $rc; }
  python -c "import json;d=json.load(open('$O/b_$name.json'));l=d['lp'];print('$name', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], l['root_iters'])"
}
run default NEP_X=0 || exit 1
run art020 NEP_RESTART=0.2,0.8,0.2 || exit 1
run art050 NEP_RESTART=0.2,0.8,0.5 || exit 1
run suff03 NEP_RESTART=0.3,0.9,0.36 || exit 1
run smooth03 NEP_OMEGA_SMOOTH=0.3 || exit 1
run smooth07 NEP_OMEGA_SMOOTH=0.7 || exit 1
BARGS="--warm-omega-floor 8" run floor8 NEP_X=0 || exit 1
BARGS="--warm-omega-floor -1" run nofloor NEP_X=0 || exit 1
BARGS="--check-every 32" run ce32 NEP_X=0 || exit 1
BARGS="--check-every 8" run ce8 NEP_X=0 || exit 1
