#!/bin/bash
# round 2, call AQ: primal feasibility polishing (step 1, warm-started LPs): bench seeds 0/1, then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02aq; mkdir -p $O
timeout -k 10 300 python -u bench.py --cpu-budget 0 --bnb-seconds 20 > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.log; exit $rc; }
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3)); print(d['bnb'])"
timeout -k 10 300 python -u bench.py --seed 1 --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/bench_s1.json 2> $O/bench_s1.log
rc=$?; echo "bench s1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench_s1.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -s > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -20; grep -c UNCERTIFIED $O/pytest_gpu.log
