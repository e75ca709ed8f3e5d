#!/bin/bash
# Round 5: per-node-LP records of the replay bench (bench.py --dump) under both root regimes
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_dump}; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1"
timeout -k 10 240 python -u bench.py $Q --dump "$O/rec_slow.json" > "$O/b_slow.json" 2> "$O/b_slow.err" || exit $?
NEP_ETA_SCALE=0.9999999999997 timeout -k 10 240 python -u bench.py $Q --dump "$O/rec_fast.json" > "$O/b_fast.json" 2> "$O/b_fast.err" || exit $?
echo dump ok
