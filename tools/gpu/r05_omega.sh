#!/bin/bash
# Round 5: the replay bench under the two root regimes (NEP_ETA_SCALE picks the root trajectory: 1 -> the slow
# root, omega ~4e-6; 0.9999999999997 -> the fast one, omega ~1.6e-5) x warm primal-weight floors
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_omega}; mkdir -p "$O"; shift
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1"
for sc in 1 0.9999999999997; do
  for fl in "$@"; do
    NEP_ETA_SCALE=$sc timeout -k 10 240 python -u bench.py $Q --warm-omega-floor $fl > "$O/b_${sc}_${fl}.json" 2> "$O/b_${sc}_${fl}.err" || exit $?
    python - "$O/b_${sc}_${fl}.json" "$sc" "$fl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); lp = d.get("lp", {})
print("scale", sys.argv[2], "floor", sys.argv[3], "value", round(d["value"], 3), "root_s", lp.get("root_seconds"),
      "root_iters", lp.get("root_iters"), "mean_iters", round(lp.get("mean_iters"), 1), "cert", lp.get("certified"), "done", lp.get("completed"),
      {k: v for k, v in lp.items() if "warm" in k}, flush=True)
PY
  done
done
