#!/usr/bin/env python3
"""Dev probe (GPU box): the leaves a golden flow's step-2 B&B leaves unresolved (uncertified after their
retry), re-solved by HiGHS on the reference formulation (oracle/) — infeasible, or their LP value —
with the engine's residual / bound at the stop.

  python3 tools/unresolved_probe.py syn_6x4_s1_r0.3_NeptuneMinDelay
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    import core.solvers as S
    from core.engine import bnb as B
    from core.engine.lp import LP_OPTIMAL
    from core.utils import data_to_solver_input
    from golden_util import payload
    from oracle.formulation import build_model
    from oracle.solve import solve
    name = sys.argv[1]
    rec = []
    orig = B.BranchAndBound._finish

    def finish(self, slot, node, st, obj, pobj, iters, inc):
        if node.kind == B.RETRY and st != LP_OPTIMAL:
            dg = self.lp.diag(slot)
            rec.append((self.lp.step, node.idx.copy(), node.val.copy(), st, obj, pobj, dg["pres"], iters))
        return orig(self, slot, node, st, obj, pobj, iters, inc)

    B.BranchAndBound._finish = finish
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    solver.load_data(data)
    solver.solve()
    print(name, "score", solver.score())
    variant = {"NeptuneMinDelay": "MinDelay", "NeptuneMinUtilization": "MinUtilization",
               "NeptuneMinDelayAndUtilization": "MinDelayAndUtilization"}[p["solver"]["type"]]
    N, F = len(data.nodes), len(data.functions)
    nx = N * N * F
    for step, idx, val, st, obj, pobj, pres, iters in rec:
        if step == 1:
            continue
        m = build_model(data, variant, step=2, mode="delete" if step == 2 else "create", alpha=0.5,
                        soften_step1_sol=1.3, max_score=data.max_score,
                        prev_x=np.asarray(data.prev_x, np.float64))
        lb, ub = m["lb"].copy(), m["ub"].copy()
        lb[nx + idx] = val
        ub[nx + idx] = val
        hst, hobj, _ = solve(m, relax=True, lb=lb, ub=ub)
        print(f"  step {step} leaf: engine st {st} bound {obj:.6g} pobj {pobj:.6g} res {pres:.2e} its {iters} | "
              f"HiGHS status {hst} value {hobj}")


if __name__ == "__main__":
    main()
