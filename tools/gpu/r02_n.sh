#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02n; mkdir -p $O
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 16 --cpu-budget 0 --bnb-seconds 0 ${BARGS:-} > $O/b_$name.json 2> $O/b_$name.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 $O/b_$name.log; return $rc; }
  python -c "import json;d=json.load(open('$O/b_$name.json'));l=d['lp'];print('$name', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], l['root_iters'])"
}
run default NEP_X=0 || exit 1
run s3_9_36 NEP_RESTART=0.3,0.9,0.36 || exit 1
run s3_9_30 NEP_RESTART=0.3,0.9,0.30 || exit 1
run s4_9_36 NEP_RESTART=0.4,0.9,0.36 || exit 1
run s3_95_36 NEP_RESTART=0.3,0.95,0.36 || exit 1
run s3_8_36 NEP_RESTART=0.3,0.8,0.36 || exit 1
run s2_9_36 NEP_RESTART=0.2,0.9,0.36 || exit 1
run s3_9_42 NEP_RESTART=0.3,0.9,0.42 || exit 1
BARGS="--check-every 12" run s3_9_36_ce12 NEP_RESTART=0.3,0.9,0.36 || exit 1
BARGS="--warm-omega-floor 3" run s3_9_36_f3 NEP_RESTART=0.3,0.9,0.36 || exit 1
