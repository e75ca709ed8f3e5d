#!/bin/bash
# round 2, call AD: A/B of the sparse anchor (HEAD build / current code dense / current code sparse)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ad; mkdir -p $O
for v in head dense cur; do
  L=neptune-mip_amd/lib/variants/libneptune_lp_$v.so; [ $v = cur ] && L=neptune-mip_amd/lib/libneptune_lp.so
  NEPTUNE_LP_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 > $O/b_$v.json 2> $O/b_$v.log
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 $O/b_$v.log; exit $rc; }
  grep "root LP" $O/b_$v.log | cut -c1-200
  python -c "import json;d=json.load(open('$O/b_$v.json'));l=d['lp'];print('$v', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3), round(d['ms_per_step'],1))"
done
