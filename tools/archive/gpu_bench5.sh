#!/bin/bash
# GPU box: default bench line, then a rocprofv3 kernel-trace/stats pass over a shorter bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u bench.py > gpurun_out/bench5.json 2> gpurun_out/bench5.log
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench5.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof5 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-budget 0 > $R/gpurun_out/bench5_prof.json 2> $R/gpurun_out/bench5_prof.log
rc=$?; echo "rocprof rc=$rc"
exit $rc
