#!/bin/bash
# round 2, call AF: bench A/B — HEAD build, current code without / with the root gap polish
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02af; mkdir -p $O
run() {  # name lib args...
  local v=$1 L=$2; shift 2
  NEPTUNE_LP_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 "$@" > $O/b_$v.json 2> $O/b_$v.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/b_$v.log; return $rc; }
  grep "root" $O/b_$v.log | cut -c1-200
  python -c "import json;d=json.load(open('$O/b_$v.json'));l=d['lp'];print('$v', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3), round(d['ms_per_step'],1))"
}

run cur0 neptune-mip_amd/lib/libneptune_lp.so --root-gap-tol 0 &&
run cur8 neptune-mip_amd/lib/libneptune_lp.so --root-gap-tol 1e-8 &&
run cur9 neptune-mip_amd/lib/libneptune_lp.so --root-gap-tol 1e-9
