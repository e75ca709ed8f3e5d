#!/usr/bin/env python3
"""Dev probe (GPU box): the hard and easy warm-started children of tools/child_probe.py under
several warm-start primal-weight floors (nep_lp_opts.warm_omega_floor; PROBE_FLOORS=-1,2,4)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402

HARD = [12, 17, 26, 29, 34, 36, 37, 40]
EASY = [1, 4, 5, 7, 8, 10, 11, 13]
# (name, warm_omega_floor, warm start): -1 = no floor (the PDLP update alone)
VARIANTS = [(f"floor{f}", float(f), True) for f in os.environ.get("PROBE_FLOORS", "-1,4").split(",")]
if os.environ.get("PROBE_COLD"):
    VARIANTS.append(("cold", 0.0, False))


def main():
    a = bench.parse(sys.argv[1:])
    import torch
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    B = len(HARD)
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=B + 1)
    rr = m.solve([B], tol=a.tol, max_iters=a.root_max_iters, check_every=a.check_every)
    print(f"root st={rr['status'][0]} it={rr['iters'][0]} diag={m.diag(B)}", flush=True)
    for which, ids in (("hard", HARD), ("easy", EASY))[: int(os.environ.get("PROBE_SETS", "2"))]:
        lbs, ubs = [], []
        for k in ids:
            lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, (a.seed * 1000003) * 7919 + k)
            lbs.append(lb[0])
            ubs.append(ub[0])
        for name, floor, warm in VARIANTS:
            if warm:
                for s in range(B):
                    m.copy_state(B, s)
            t = time.perf_counter()
            r = m.solve(np.arange(B), np.array(lbs), np.array(ubs), tol=a.tol, max_iters=a.max_iters,
                        check_every=a.check_every, warm_start=warm, warm_omega_floor=floor)
            dt = time.perf_counter() - t
            om = [f"{m.diag(s)['omega']:.2g}" for s in range(B)]
            print(f"{which} {name:12s} {dt:6.2f}s st={r['status'].tolist()} it={r['iters'].tolist()} "
                  f"omega={om}", flush=True)
    m.close()


if __name__ == "__main__":
    main()
