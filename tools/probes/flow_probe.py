#!/usr/bin/env python3
"""Dev probe (GPU box): a two-step solver flow on the engine, step by step, with every step's B&B
incumbent re-solved by the oracle (HiGHS on the reference formulation, leaf = the incumbent's c and n
fixed): a certified incumbent must have the oracle's leaf value.

  python3 tools/flow_probe.py testpy NeptuneWithEFTTCMinDelayAndUtilization
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main(name, stype):
    import core.solvers as S
    from core.utils import data_to_solver_input
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve as oracle_solve
    with open(os.path.join(REPO, "tests", "golden", "inputs", name + ".json")) as fh:
        p = json.load(fh)
    p["solver"] = dict(p["solver"], type=stype)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[stype](**p["solver"].get("args", {}))
    solver.load_data(data)
    solved = solver.solve()
    print("solved", solved, "score", solver.score(), flush=True)
    od = oracle_input(p, with_db=False)
    F, N = len(data.functions), len(data.nodes)
    for k, mode in (("step2_delete", "delete"), ("step2_create", "create")):
        st = getattr(solver, k)
        r = getattr(st, "result", None)
        if r is None:
            continue
        print(k, r.as_dict(), flush=True)
        m = build_model(od, "MinDelayAndUtilization", step=2, mode=mode, alpha=0.5,
                        soften_step1_sol=p["solver"].get("args", {}).get("soften_step1_sol", 1.3),
                        max_score=float(data.max_score), prev_x=np.zeros((N, F, N)))
        stm, objm, _ = oracle_solve(m, relax=False)
        print("   oracle MIP of this step:", stm, objm, "max_score", data.max_score, flush=True)
        if r.z is not None:
            nx = N * N * F
            lb, ub = m["lb"].copy(), m["ub"].copy()
            zc = np.asarray(r.z)
            L = m["layout"]
            for a0, a1 in ((L.c0, L.c0 + F * N), (L.n0, L.n0 + N)):
                lb[a0:a1] = ub[a0:a1] = np.round(zc[a0 - nx:a1 - nx])
            st2, obj2, _ = oracle_solve(m, relax=True, lb=lb, ub=ub)
            print("   incumbent", r.objective, "oracle leaf LP", st2, obj2, "z_small", zc[:].tolist()[:40], flush=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
