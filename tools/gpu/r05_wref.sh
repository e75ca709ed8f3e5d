#!/bin/bash
# Round 5: the replay bench with warm starts banded around k x omega0 (bench --omega-ref k) under a root regime
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_wref}; SC=${2:-1}; shift 2; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1"
for k in "$@"; do
  NEP_ETA_SCALE=$SC timeout -k 10 240 python -u bench.py $Q --omega-ref $k > "$O/b_${SC}_$k.json" 2> "$O/b_${SC}_$k.err" || exit $?
  python - "$O/b_${SC}_$k.json" "$k" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); lp = d["lp"]
print("k", sys.argv[2], "value", round(d["value"], 3), "root_iters", lp["root_iters"], "mean_iters",
      round(lp["mean_iters"], 1), "cert", lp["certified"], "/", lp["completed"], "w0", lp["primal_weight0"],
      "wroot", lp["root_final_weight"], "ref", lp["omega_ref"], flush=True)
PY
done
