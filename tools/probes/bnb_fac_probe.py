#!/usr/bin/env python3
"""Dev probe (GPU box): the product B&B with the facility-relaxation bound model against the
single-model search, time-limited, at BASELINE configs 2-4: status, incumbent, bound, gap, node-LP mix.

  python3 tools/bnb_fac_probe.py 64x32:20 256x128:40 512x256:60   [MODES=two,one]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]


def run(N, F, secs, two, knobs):
    from core.engine.bnb import BranchAndBound
    from core.engine.lp import LPModel, RELAX_FACILITY
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    p = synthetic_payload(N, F, seed=int(os.environ.get("SEED", "0")))
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    bm = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=33, relaxation=RELAX_FACILITY) if two else None
    try:
        t0 = time.time()
        res = BranchAndBound(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                             batch=32, tol=1e-6, time_limit=secs, root_max_iters=400000,
                             upper_bound=ub * (1 + 1e-6) + 1e-6, repair=st1.routing_repair(m.layout()),
                             node_max_iters=1024, bound_lp=bm, log=lambda s: print("   ", s, flush=True),
                             primal=st1.primal_heuristic(m.layout(), m.row_map()) if os.environ.get("PRIMAL", "1") == "1" else None,
                             **knobs).solve()
    finally:
        m.close()
        if bm is not None:
            bm.close()
    d = res.as_dict()
    gap = None if res.objective is None else (res.objective - res.bound) / max(1.0, abs(res.objective))
    print(f"{N}x{F} {'two' if two else 'one'} {knobs}: {res.status} inc {res.objective} bound {res.bound} gap {gap} "
          f"nodes {res.nodes} leaves {res.leaves} lps {res.lps} {time.time() - t0:.1f}s", flush=True)
    print("   mix", json.dumps({k: d[k] for k in ("lp_status_kind", "timing", "lp_iters_p50_p90_p99_max")}), flush=True)


def main():
    modes = os.environ.get("MODES", "two,one").split(",")
    knobs = json.loads(os.environ.get("KNOBS", "{}"))
    for arg in sys.argv[1:]:
        size, secs = arg.split(":")
        N, F = (int(t) for t in size.split("x"))
        for mode in modes:
            run(N, F, float(secs), mode == "two", knobs)


if __name__ == "__main__":
    main()
