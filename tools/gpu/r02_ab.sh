#!/bin/bash
# round 2, call AB (HEAD snapshot after the step-2 work): full GPU tests, smoke, bench (default), kernel-trace profile
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf -s > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -20
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['lp'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3)); print(d['bnb']); print(d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.log
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $O/prof > $O/kernel_stats_by_slots.csv; head -8 $O/kernel_stats_by_slots.csv | cut -c1-150
