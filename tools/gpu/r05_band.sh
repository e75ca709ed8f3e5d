#!/bin/bash
# Round 5: the replay bench with an absolute warm-start primal-weight band (NEP_WARM_OMEGA_ABS=lo,hi) against the
# parent-relative default, under a root regime (NEP_ETA_SCALE); per-LP records kept
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_band}; SC=${2:-1}; shift 2; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1"
for band in "$@"; do
  t=$(echo "$band" | tr ',' '_')
  if [ "$band" = none ]; then unset NEP_WARM_OMEGA_ABS; else export NEP_WARM_OMEGA_ABS=$band; fi
  NEP_ETA_SCALE=$SC timeout -k 10 240 python -u bench.py $Q --dump "$O/rec_${SC}_$t.json" > "$O/b_${SC}_$t.json" 2> "$O/b_${SC}_$t.err" || exit $?
  python - "$O/b_${SC}_$t.json" "$band" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); lp = d["lp"]
print("band", sys.argv[2], "value", round(d["value"], 3), "root_iters", lp["root_iters"], "mean_iters",
      round(lp["mean_iters"], 1), "cert", lp["certified"], "/", lp["completed"], flush=True)
PY
done
