#!/bin/bash
# Round 4: root polishing (cold root, polish_after 256 / 1024) vs none: root seconds and the replay rate
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_rootpol}; mkdir -p "$O"
for pa in 0 256 1024; do
  timeout -k 10 300 python -u bench.py --steps 6 --root-polish-after $pa --native-steps 0 --children-steps 12 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_pa$pa.json" 2> "$O/bench_pa$pa.err"
  rc=$?; echo "bench pa=$pa rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_pa$pa.json'));print(d['value'], d['lp']['certified'], d['lp']['root_iters'], d['lp']['root_seconds'], d['children_stream']['value'])"
  [ $rc -eq 0 ] || exit $rc
done
