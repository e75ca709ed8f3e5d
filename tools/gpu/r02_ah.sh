#!/bin/bash
# round 2, call AH: bench LP/s over instance seeds 1, 2 for HEAD kernels (va), node-pass prefetch (vc), current code
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ah; mkdir -p $O
run() {
  local v=$1 L=$2; shift 2
  NEPTUNE_LP_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --steps 4 --cpu-budget 0 --bnb-seconds 0 --root-gap-tol 0 "$@" > $O/b_$v.json 2> $O/b_$v.log
  local rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/b_$v.log; return $rc; }
  grep "root LP" $O/b_$v.log | cut -c20-200
  python -c "import json;d=json.load(open('$O/b_$v.json'));l=d['lp'];print('$v', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],4), round(d['ms_per_step'],1))"
}
for s in 1 2; do
run va_s$s neptune-mip_amd/lib/variants/libneptune_lp_va.so --seed $s &&
run vc_s$s neptune-mip_amd/lib/variants/libneptune_lp_vc.so --seed $s &&
run cur_s$s neptune-mip_amd/lib/libneptune_lp.so --seed $s || exit 1
done
