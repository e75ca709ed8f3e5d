#!/bin/bash
# round 2, call AU: bench at the closing head (seeds 0 and 1) and smoke
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02au; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], round(d['roofline']['frac'],3), d['roofline']['avg_launch_ms']); print(d['bnb']); print(d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 300 python -u bench.py --seed 1 --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/bench_s1.json 2> $O/bench_s1.log
rc=$?; echo "bench s1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench_s1.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], round(d['roofline']['frac'],3))"
