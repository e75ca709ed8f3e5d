#!/bin/bash
# Round 5: the warm-start reference weight on seed 1's replay and in the product B&B (tools/bnb_ab.py, BNB_WREF)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_wref2}; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1 --seed 1"
for k in 0 8; do
  timeout -k 10 300 python -u bench.py $Q --omega-ref $k > "$O/s1_$k.json" 2> "$O/s1_$k.err" || exit $?
  python - "$O/s1_$k.json" "$k" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); lp = d["lp"]
print("seed1 k", sys.argv[2], "value", round(d["value"], 3), "root_iters", lp["root_iters"], "root_s", round(lp["root_seconds"], 2),
      "mean_iters", round(lp["mean_iters"], 1), "cert", lp["certified"], "/", lp["completed"], flush=True)
PY
done
for k in 0 8; do
  for sz in "256 128 20" "512 256 60"; do
    BNB_WREF=$k timeout -k 10 300 python -u tools/bnb_ab.py $sz > "$O/bnb_${k}_${sz// /_}.json" 2> "$O/bnb_${k}_${sz// /_}.err" || exit $?
    python - "$O/bnb_${k}_${sz// /_}.json" "$k $sz" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("bnb", sys.argv[2], d["status"], "obj", d["objective"], "bound", d["bound"], "nodes", d["nodes"], "lps", d["lps"],
      "cert", d["certified"], "iters_p50", d["lp_iters_p50_p90_p99_max"], flush=True)
PY
  done
done
