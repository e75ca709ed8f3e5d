#!/bin/bash
# Round 5: root LP iterations under eta perturbations (tools/root_chaos_probe.py) for primal-weight smoothing values
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_rootw}; shift; mkdir -p "$O"
for seed in 0 1; do
  for th in "$@"; do
    echo "== seed $seed NEP_OMEGA_SMOOTH=$th"
    ROOT_SEED=$seed NEP_OMEGA_SMOOTH=$th timeout -k 10 300 python -u tools/root_chaos_probe.py 1 0.9999999999997 1.000000001 0.999999 1.001 > "$O/s${seed}_$th.log" 2>&1 || exit $?
    grep scale "$O/s${seed}_$th.log" | cut -c1-120
  done
done
