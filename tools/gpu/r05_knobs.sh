#!/bin/bash
# Round 5: replay-bench knob sweep (each argument: [ENV=VAL[;ENV=VAL]@]comma-separated bench.py arguments, "-" = defaults)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_knobs}; shift; mkdir -p "$O"
Q="--native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 --steps 12 --warmup 1"
i=0
for args in "$@"; do
  i=$((i+1)); E=""
  case $args in *@*) E=${args%%@*}; args=${args#*@} ;; esac
  A=""; [ "$args" = "-" ] || A=${args//,/ }
  env ${E//;/ } timeout -k 10 240 python -u bench.py $Q $A > "$O/k$i.json" 2> "$O/k$i.err" || exit $?
  python - "$O/k$i.json" "$E@$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); lp = d["lp"]; w = lp["iters_by_warm_source_rank0"]
print(sys.argv[2], "value", round(d["value"], 3), "mean_iters", round(lp["mean_iters"], 1), "cert", lp["certified"], "/",
      lp["completed"], "parent", w["parent"], "root", w["root"], "frac", round(d["roofline"]["frac"], 4), flush=True)
PY
done
