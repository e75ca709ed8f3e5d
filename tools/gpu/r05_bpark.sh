#!/bin/bash
# Round 5: parked parents on the product search's bound model (BNB_PARK extra slots; tools/bnb_ab.py product mode)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_bpark}; shift; mkdir -p "$O"
export BNB_MODE=product
for pk in "$@"; do
  for sz in "64 32 10" "256 128 20" "512 256 60"; do
    BNB_PARK=$pk timeout -k 10 300 python -u tools/bnb_ab.py $sz > "$O/bnb_${pk}_${sz// /_}.json" 2> "$O/bnb_${pk}_${sz// /_}.err" || exit $?
    python - "$O/bnb_${pk}_${sz// /_}.json" "park $pk $sz" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
inc, b = d["objective"], d["bound"]; t = d["timing"]
print(sys.argv[2], d["status"], "obj", inc, "bound", b, "gap", None if inc is None else round((inc - b) / max(1.0, abs(inc)), 5),
      "nodes", d["nodes"], "lps", d["lps"], "iters", d["lp_iters_p50_p90_p99_max"], "host", round(1 - t["advance"] / d["seconds"], 3),
      "native", d.get("native"), flush=True)
PY
  done
done
