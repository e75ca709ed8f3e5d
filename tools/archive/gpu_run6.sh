#!/bin/bash
# GPU box: parity tests, bench line, rocprofv3 kernel stats, PMC traffic passes for the bench kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu6.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/bench6.json 2> gpurun_out/bench6.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof6 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-budget 0 > $R/gpurun_out/bench6_prof.json 2> $R/gpurun_out/bench6_prof.log
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch6 -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/pmc_fetch6.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write6 -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/pmc_write6.log 2>&1
rc=$?; echo "pmc write rc=$rc"
exit $rc
