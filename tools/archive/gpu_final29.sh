#!/bin/bash
# GPU box (round-1 closing snapshot): parity suite, smoke, PMC traffic passes for x_pass, the
# default bench line reading that traffic (CPU baseline included), and a rocprofv3
# kernel-trace/stats pass over a shorter bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r29
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 $R/tools/traffic.py run > $O/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 $R/tools/traffic.py run > $O/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
python3 tools/traffic.py summarize $O/pmc_fetch $O/pmc_write > $O/traffic.json
rc=$?; echo "summarize rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --traffic $O/traffic.json > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; cat $O/bench.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $O/prof -o run -- python3 $R/bench.py --steps 8 --cpu-budget 0 > $O/bench_prof.json 2> $O/bench_prof.log
rc=$?; echo "rocprof rc=$rc"
exit $rc
