#!/bin/bash
# round 2, call J: node_pass over 16-node workgroups + working-set-dependent nt: GPU tests, A/B bench, root profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -30
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
for v in default plain; do
  if [ $v = default ]; then lib=neptune-mip_amd/lib/libneptune_lp.so; else lib=neptune-mip_amd/lib/variants/libneptune_lp_$v.so; fi
  NEPTUNE_LP_LIB=$PWD/$lib timeout -k 10 240 python -u bench.py --steps 12 --cpu-budget 0 --bnb-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.log
  rc=$?; echo "bench $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['value'],1), d['lp']['certified'], d['lp']['completed'], round(d['lp']['mean_iters'],1), d['lp']['root_iters'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
  grep "root LP" $O/bench_$v.log
done
