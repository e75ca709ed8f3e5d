#!/bin/bash
# round 2, call A: GPU tests on the new build, x_pass A/B variants, tail probe
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02a; mkdir -p $O
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; ok $rc || exit $rc
for v in base nt f16 default; do
  if [ $v = default ]; then lib=neptune-mip_amd/lib/libneptune_lp.so; else lib=neptune-mip_amd/lib/variants/libneptune_lp_$v.so; fi
  NEPTUNE_LP_LIB=$PWD/$lib timeout -k 10 180 python -u bench.py --steps 12 --cpu-budget 0 > $O/bench_$v.json 2> $O/bench_$v.log
  rc=$?; echo "bench $v rc=$rc"; ok $rc || exit $rc
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['value'],1), d['lp']['certified'], d['lp']['completed'], d['lp']['mean_iters'], d['roofline']['avg_launch_ms'], round(d['roofline']['frac'],3))"
done
timeout -k 10 300 python -u tools/tail_probe.py --probe-nodes 192 > $O/tail_probe.log 2>&1
rc=$?; echo "tail rc=$rc"; tail -40 $O/tail_probe.log
exit $rc
