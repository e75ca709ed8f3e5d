#!/bin/bash
# round 2, call AG: isolate the root-LP convergence change: HEAD kernels (va), + scalar_pass reduction (vb),
# + node_pass prefetch (vc), current code (cur); root iterations / gap / children certified per build
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ag; mkdir -p $O
run() {
  local v=$1 L=$2; shift 2
  NEPTUNE_LP_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --steps 4 --cpu-budget 0 --bnb-seconds 0 --root-gap-tol 0 "$@" > $O/b_$v.json 2> $O/b_$v.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/b_$v.log; return $rc; }
  grep "root" $O/b_$v.log | cut -c1-200
  python -c "import json;d=json.load(open('$O/b_$v.json'));l=d['lp'];print('$v', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3), round(d['ms_per_step'],1))"
}
run va neptune-mip_amd/lib/variants/libneptune_lp_va.so &&
run vb neptune-mip_amd/lib/variants/libneptune_lp_vb.so &&
run vc neptune-mip_amd/lib/variants/libneptune_lp_vc.so
