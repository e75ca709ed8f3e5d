#!/usr/bin/env python3
"""Dev probe (GPU box): iteration statistics of the bench's first `PROBE_N` warm-started child
LPs (rank 0's stream seeds) under several warm-start primal-weight floors (PROBE_FLOORS)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:])
    import torch
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    n_probe = int(os.environ.get("PROBE_N", "96"))
    floors = [float(f) for f in os.environ.get("PROBE_FLOORS", "-1,2,4,8").split(",")]
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    B = a.batch
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=B + 1)
    rr = m.solve([B], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every)
    print(f"root st={rr['status'][0]} it={rr['iters'][0]}", flush=True)
    nodes = []
    for k in range(n_probe):
        lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, (a.seed * 1000003) * 7919 + k)
        nodes.append((lb[0], ub[0]))
    for fl in floors:
        its, sts = [], []
        t = time.perf_counter()
        for b0 in range(0, n_probe, B):
            nb = min(B, n_probe - b0)
            for s in range(nb):
                m.copy_state(B, s)
            r = m.solve(np.arange(nb), np.array([n[0] for n in nodes[b0:b0 + nb]]),
                        np.array([n[1] for n in nodes[b0:b0 + nb]]), tol=a.tol, max_iters=a.max_iters,
                        check_every=a.check_every, warm_start=True, warm_omega_floor=fl)
            its += r["iters"].tolist()
            sts += r["status"].tolist()
        its, sts = np.array(its), np.array(sts)
        slow = np.argsort(-its)[:8]
        print(f"floor {fl:5}: {time.perf_counter() - t:6.2f}s total_it={its.sum()} certified={int((sts == 0).sum())}/"
              f"{n_probe} >1000: {int((its > 1000).sum())} p50/p90/max {np.percentile(its, [50, 90, 100]).astype(int).tolist()} "
              f"slowest {[(int(i), int(its[i]), int(sts[i])) for i in slow]}", flush=True)
    m.close()


if __name__ == "__main__":
    main()
