#!/bin/bash
# Round 4: replay stream vs certificate interval / node-LP iteration limit
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_mi}; mkdir -p "$O"
for cfg in "48 12288" "48 16384" "48 32768"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 6 --check-every $1 --max-iters $2 --native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_$1_$2.json" 2> "$O/bench_$1_$2.err"
  rc=$?; echo "bench ce=$1 mi=$2 rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_$1_$2.json'));print(d['value'], d['lp']['certified'], d['lp']['completed'], d['lp']['mean_iters'], d['roofline']['frac'])"
  [ $rc -eq 0 ] || exit $rc
done
