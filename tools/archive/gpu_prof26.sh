#!/bin/bash
# GPU box: PMC traffic passes for the bench kernel, then the bench line (with CPU baseline) reading
# that traffic, then a rocprofv3 kernel-trace/stats pass (csv + rocpd) over a shorter bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r26
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r26/pmc_fetch -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/r26/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r26/pmc_write -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/r26/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
python3 tools/traffic.py summarize gpurun_out/r26/pmc_fetch gpurun_out/r26/pmc_write > gpurun_out/r26/traffic.json
rc=$?; echo "summarize rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --traffic gpurun_out/r26/traffic.json > gpurun_out/r26/bench.json 2> gpurun_out/r26/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $R/gpurun_out/r26/prof -o run -- python3 $R/bench.py --steps 8 --cpu-budget 0 > $R/gpurun_out/r26/bench_prof.json 2> $R/gpurun_out/r26/bench_prof.log
rc=$?; echo "rocprof rc=$rc"
exit $rc
