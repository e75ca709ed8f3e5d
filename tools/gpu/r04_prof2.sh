#!/bin/bash
# Round 4: rocprofv3 kernel trace of the bench at its closing defaults (check 48, limit 8192; short run)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_prof2}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --steps 4 --native-steps 0 --children-steps 4 --bnb-seconds 0 --cpu-budget 0 > "$O/prof_bench.json" 2> "$O/prof_bench.err"
rc=$?; echo "rocprof rc=$rc"; exit $rc
