#!/usr/bin/env python3
"""Dev probe (GPU box): a golden step-1 search that ends LIMIT — every leaf / retry LP that does not certify,
with the engine's diagnostics, against HiGHS on the same box of the reference formulation (oracle/).

  python3 tools/leaf_limit_probe.py testpy
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    import core.solvers as S
    from core.engine import bnb as B
    from core.utils import data_to_solver_input
    from golden_util import payload
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve as oracle_solve
    name = sys.argv[1]
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    od = oracle_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    step1 = solver.step1
    step1.load_data(data)
    args = p["solver"].get("args", {})
    ref = build_model(od, step1.VARIANT, step=1, alpha=args.get("alpha", 0.5))
    N, F = len(data.nodes), len(data.functions)
    nx = N * N * F
    seen = []
    orig = B.BranchAndBound._finish

    def rec(self, eng, slot, node, st, obj, pobj, iters, inc):
        if node.kind in (B.LEAF, B.RETRY) and st != 0:
            d = eng.lp.diag(slot)
            seen.append((B._KIND_NAME[node.kind], st, obj, pobj, iters, d, np.asarray(node.idx), np.asarray(node.val)))
        return orig(self, eng, slot, node, st, obj, pobj, iters, inc)
    B.BranchAndBound._finish = rec
    step1.solve()
    r = step1.result
    print(name, r.status, r.objective, r.bound, r.as_dict()["lp_status_kind"], flush=True)
    for kind, st, obj, pobj, iters, d, idx, val in seen:
        lb, ub = ref["lb"].copy(), ref["ub"].copy()
        lb[nx + idx] = val
        ub[nx + idx] = val
        hst, hv, _ = oracle_solve(ref, relax=True, lb=lb, ub=ub)
        opened = idx[val > 0.5].tolist()
        print(f"  {kind}: status {st} obj {obj:.9g} pobj {pobj:.9g} iters {iters} pres {d['pres']:.2e} gap {d['gap']:.2e} "
              f"omega {d['omega']:.3g} | HiGHS status {hst} value {hv} | open {opened}", flush=True)


if __name__ == "__main__":
    main()
