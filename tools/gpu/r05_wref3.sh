#!/bin/bash
# Round 5: the warm-start reference weight in the product's two-model step-1 search (tools/bnb_ab.py, BNB_MODE=product)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_wref3}; mkdir -p "$O"
export BNB_MODE=product
for k in 0 8; do
  for sz in "256 128 20" "512 256 60"; do
    BNB_WREF=$k timeout -k 10 300 python -u tools/bnb_ab.py $sz > "$O/bnb_${k}_${sz// /_}.json" 2> "$O/bnb_${k}_${sz// /_}.err" || exit $?
    python - "$O/bnb_${k}_${sz// /_}.json" "$k $sz" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
inc, b = d["objective"], d["bound"]
print("bnb", sys.argv[2], d["status"], "obj", inc, "bound", b, "gap", None if inc is None else (inc - b) / max(1.0, abs(inc)),
      "nodes", d["nodes"], "lps", d["lps"], "cert", d["certified"], "iters", d["lp_iters_p50_p90_p99_max"], flush=True)
PY
  done
done
