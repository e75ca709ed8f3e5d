#!/usr/bin/env python3
"""Dev probe (GPU box): the capacity-greedy heuristic at the facility root of a synthetic instance — leaves
found, open nodes, estimate and seconds per (new_pen, tries), and whether each passes check_placement.

  python3 tools/greedy_probe.py 512x256 256x128
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402


def main():
    from core.engine.heuristics import capacity_greedy
    from core.engine.lp import LPModel, RELAX_FACILITY
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    for size in sys.argv[1:]:
        N, F = (int(t) for t in size.split("x"))
        data = data_to_solver_input(synthetic_payload(N, F, seed=0), with_db=False)
        st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
        st1.load_data(data)
        bm = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=2, relaxation=RELAX_FACILITY)
        t0 = time.time()
        r = bm.solve([0], tol=1e-6, max_iters=400000, check_every=12, bound_res=1e-2, gap_tol=1e-4)
        z, _ = bm.solution(0, dense_x=False)
        flow = bm.flows([0])[0]
        L = bm.layout()
        n0, n1 = L["n"]
        print(f"{size}: fac root status {r['status'][0]} obj {r['obj'][0]:.6g} {time.time() - t0:.1f}s sum n {z[n0:n1].sum():.2f}",
              flush=True)
        wts = st1.objective_weights()
        d = data
        for pen in (0.5, 1.0, 2.0, 4.0):
            t1 = time.time()
            out = capacity_greedy(d.workload_matrix, d.node_delay_matrix, d.core_per_req_matrix, d.node_cores_matrix,
                                  d.function_memory_matrix, d.node_memory_matrix, z[n0:n1], flow=flow, tries=4,
                                  node_cost=wts[0], delay_coef=wts[1], new_pen=pen)
            res = [(int(C.sum()), int(n.sum()), round(est, 5)) for C, n, est, _ in out]
            print(f"   new_pen {pen}: {res} {time.time() - t1:.2f}s", flush=True)
        bm.close()


if __name__ == "__main__":
    main()
