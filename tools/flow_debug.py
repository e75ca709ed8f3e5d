#!/usr/bin/env python3
"""Dev probe (GPU box): one golden solver flow with every step's B&B summary (status, objective, bound,
LP mix) printed, to see which step of NeptuneBase.solve (neptune.py:18-30) ends where.

  python3 tools/flow_debug.py syn_6x4_s1_r0.3_NeptuneMinDelay
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]


def main():
    import core.solvers as S
    from core.utils import data_to_solver_input
    from golden_util import golden, payload
    for name in sys.argv[1:]:
        p = payload(name)
        data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
        solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
        solver.load_data(data)
        solver.solve()
        print(name, "score", solver.score(), "reference", golden()[name]["response"]["score"])
        for k in ("step1", "step2_delete", "step2_create"):
            st = getattr(solver, k, None)
            r = getattr(st, "result", None)
            if r is not None:
                d = r.as_dict()
                print(" ", k, json.dumps({q: d[q] for q in ("status", "objective", "bound", "nodes", "leaves", "lps",
                                                           "certified", "unresolved", "lp_status", "seconds")},
                                         default=str))


if __name__ == "__main__":
    main()
