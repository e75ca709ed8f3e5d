#!/bin/bash
# Round 5 A/B: the replay bench (CPU baseline / B&B / native / children skipped) on the current build and on a
# variant library (NEPTUNE_LP_LIB), same arguments
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_ab}; V=${2:-lib/variants/libneptune_lp_r04head.so}; shift 2; ARGS="$*"
mkdir -p "$O"
export TMPDIR=/tmp
Q="--cpu-budget 0 --bnb-seconds 0 --native-steps 0 --children-steps 0 --steps 12 $ARGS"
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
        echo "   rc=$rc"; grep "^{" "$O/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); lp=d['lp']; print('value', round(d['value'],3), 'frac', round(d['roofline']['frac'],4), 'launch_ms', round(d['roofline']['avg_launch_ms'],4), 'lps/launch', round(d['roofline']['algorithmic_bytes_per_launch']/d['roofline']['algorithmic_bytes_per_lp_iter'],2), 'mean_iters', round(lp['mean_iters']), 'cert', lp['certified'], 'root_iters', lp['root_iters'], lp['root_seconds'])"
        [ $rc -eq 0 ] || exit $rc; }
run bench_cur 300 python -u bench.py $Q
NEPTUNE_LP_LIB=neptune-mip_amd/$V run bench_var 300 python -u bench.py $Q
