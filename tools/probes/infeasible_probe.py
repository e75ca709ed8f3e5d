#!/usr/bin/env python3
"""Dev probe (GPU box): soundness of the engine's infeasibility verdicts.  Runs the product B&B (step 1
MDU, synthetic N x F, time-limited), records the node boxes whose LP the engine ended NEP_LP_INFEASIBLE
after iterating (the Farkas test; presolve rejections are not counted), and re-solves a sample of them
with HiGHS on the reference formulation (oracle/).  Every one must be infeasible there.

  python3 tools/infeasible_probe.py 64 32 15 [sample]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    from core.engine import bnb as B
    from core.engine.lp import LPModel, LP_INFEASIBLE
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve
    N, F, secs = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    sample = int(sys.argv[4]) if len(sys.argv) > 4 else 40
    p = synthetic_payload(N, F, seed=0)
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    rec = []
    orig = B.BranchAndBound._finish

    def finish(self, slot, node, st, obj, pobj, iters, inc):
        if st == LP_INFEASIBLE:
            rec.append((node.idx.copy(), node.val.copy(), iters, B._KIND_NAME[node.kind]))
        return orig(self, slot, node, st, obj, pobj, iters, inc)

    B.BranchAndBound._finish = finish
    res = B.BranchAndBound(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=32,
                           tol=1e-6, time_limit=secs, upper_bound=ub * (1 + 1e-6) + 1e-6).solve()
    m.close()
    print(f"{N}x{F}: B&B {res.status} lps {res.lps} engine-infeasible {len(rec)}", flush=True)
    mdl = build_model(oracle_input(p, with_db=False), "MinDelayAndUtilization", step=1, alpha=0.5)
    nx = N * N * F
    rng = np.random.default_rng(0)
    pick = rng.choice(len(rec), size=min(sample, len(rec)), replace=False) if rec else []
    bad = 0
    for t in pick:
        idx, val, iters, kind = rec[t]
        lb, ubb = mdl["lb"].copy(), mdl["ub"].copy()
        lb[nx + idx] = val
        ubb[nx + idx] = val
        st, obj, _ = solve(mdl, relax=True, lb=lb, ub=ubb)
        bad += st != 2
        print(f"  {kind} ({len(idx)} fixings, {iters} its): HiGHS status {st} value {obj}", flush=True)
    print(f"checked {len(pick)}: HiGHS-feasible among them (false infeasibility) {bad}")


if __name__ == "__main__":
    main()
