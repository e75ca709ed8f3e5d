#!/bin/bash
# Round 5: replay-bench launch time against the per-slot stride padding (NEP_SLOT_PAD floats) and slot-pool size
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_pad}; shift; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 8 --warmup 1"
for spec in "$@"; do
  pad=${spec%%:*}; park=${spec##*:}; oa=1
  case $pad in oa*) oa=${pad#oa}; pad=0 ;; esac
  NEP_SLOT_OVERALLOC=$oa NEP_SLOT_PAD=$pad timeout -k 10 240 python -u bench.py $Q --park $park > "$O/p_${pad}_${oa}_${park}.json" 2> "$O/p_${pad}_${oa}_${park}.err" || exit $?
  python - "$O/p_${pad}_${oa}_${park}.json" "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print("pad:park", sys.argv[2], "value", round(d["value"], 3), "launch_ms", round(r["avg_launch_ms"], 4), "frac", round(r["frac"], 4),
      "iters", d["lp"]["iterations"], flush=True)
PY
done
