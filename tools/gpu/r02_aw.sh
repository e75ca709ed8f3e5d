#!/bin/bash
# round 2, call AW: closing snapshot at the final head (certificate every 12) — smoke, default bench (CPU baseline + product B&B), kernel-trace
# profile, PMC traffic and SQ counters of the steady x_pass
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02aw; mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], d['roofline']); print(d['bnb']); print(d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.log
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py /tmp/prof > $O/kernel_stats_by_slots.csv; head -8 $O/kernel_stats_by_slots.csv | cut -c1-150
cp /tmp/prof/*/*stats.csv $O/ 2>/dev/null; ls /tmp/prof
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o run -- python3 tools/traffic.py run > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o run -- python3 tools/traffic.py run > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic.py summarize /tmp/pmc_fetch /tmp/pmc_write > $O/traffic.json; cat $O/traffic.json
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d /tmp/pmc_sq -o run -- python3 tools/traffic.py run > $O/pmc_sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic.py sq /tmp/pmc_sq > $O/sq.json; cat $O/sq.json
timeout -k 10 300 python -u bench.py --seed 1 --cpu-budget 0 --bnb-seconds 0 --root-max-iters 1000000 > $O/bench_s1.json 2> $O/bench_s1.log
rc=$?; echo "bench s1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench_s1.json'));print(round(d['value'],1), d['ms_per_step'], d['lp'], round(d['roofline']['frac'],3))"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -s > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -20
