#!/bin/bash
# GPU box: parity tests, bench line, rocprofv3 kernel stats, PMC traffic passes for the bench kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 360 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu7.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu7.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u bench.py > gpurun_out/bench7.json 2> gpurun_out/bench7.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof7 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-budget 0 > $R/gpurun_out/bench7_prof.json 2> $R/gpurun_out/bench7_prof.log
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch7 -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/pmc_fetch7.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write7 -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/pmc_write7.log 2>&1
rc=$?; echo "pmc write rc=$rc"
exit $rc
