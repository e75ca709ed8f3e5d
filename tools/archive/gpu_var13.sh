#!/bin/bash
# GPU box: bench with the default engine vs the no-prefetch variant library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-default nopf}; do
  if [ $v = default ]; then unset NEPTUNE_LP_LIB; else export NEPTUNE_LP_LIB=$GRAFT_REPO_ROOT/neptune-mip_amd/lib/variants/libneptune_lp_$v.so; fi
  timeout -k 10 200 python -u bench.py --cpu-budget 0 > gpurun_out/b13_$v.json 2> gpurun_out/b13_$v.log
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep "root LP" gpurun_out/b13_$v.log
  python -c "import json;d=json.load(open('gpurun_out/b13_$v.json'));print(d['value'],d['lp']['certified'],d['lp']['iterations'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'],d['roofline']['algorithmic_bytes_per_launch']/55.5e6)"
done
