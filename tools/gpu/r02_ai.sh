#!/bin/bash
# round 2, call AI: why node LPs stall (seed 1): tail probe diagnostics; the same stream at tol 1e-5 / 1e-4
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ai; mkdir -p $O
timeout -k 10 300 python -u tools/tail_probe.py --seed 1 --probe-nodes 32 --root-max-iters 1000000 > $O/tail_s1.log 2>&1
rc=$?; echo "tail rc=$rc"; grep -v "amdgpu\|Initializ" $O/tail_s1.log | cut -c1-330 | tail -45; [ $rc -eq 0 ] || exit $rc
for t in 1e-5 1e-4; do
  timeout -k 10 240 python -u bench.py --steps 4 --cpu-budget 0 --bnb-seconds 0 --root-gap-tol 0 --seed 1 --tol $t --root-max-iters 1000000 > $O/b_$t.json 2> $O/b_$t.log
  rc=$?; [ $rc -eq 0 ] || { echo "tol $t rc=$rc"; tail -3 $O/b_$t.log; exit $rc; }
  grep "root LP" $O/b_$t.log | cut -c20-200
  python -c "import json;d=json.load(open('$O/b_$t.json'));l=d['lp'];print('tol $t', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['ms_per_step'],1))"
done
