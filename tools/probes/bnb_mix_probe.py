#!/usr/bin/env python3
"""Dev probe (GPU box): the product B&B's node-LP mix.  Runs core.engine.bnb on the bench's synthetic
instance (step-1 MDU, time-limited) and records every finished node LP: kind (node / leaf / retry),
depth, fixings, status, iterations, and for LPs that stop at the node-LP limit the certificate's two
sides at the stop (primal residual of the repaired point, gap to the bound).  Prints the mix and the
limit LPs' residual / gap distribution, i.e. whether they lack feasibility or optimality.

  python3 tools/bnb_mix_probe.py [N F seconds]        (default 256 128 20)
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402


def main():
    from core.engine import bnb as B
    from core.engine.lp import LPModel, LP_BOUND, LP_ITERATION_LIMIT
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F, secs = (int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (256, 128, 20.0)
    p = synthetic_payload(N, F, seed=0)
    data = data_to_solver_input(p, with_db=False)
    alpha = p["solver"]["args"]["alpha"]
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=alpha, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=34)
    rec = []
    orig = B.BranchAndBound._finish

    def finish(self, slot, node, st, obj, pobj, iters, inc):
        row = dict(kind=B._KIND_NAME[node.kind], depth=node.depth, nfix=len(node.idx), st=st, iters=iters)
        if st in (LP_ITERATION_LIMIT, LP_BOUND):
            dg = self.lp.diag(slot)
            row.update(pres=dg["pres"], gap=(dg["pobj"] - dg["best_lagr"]) / max(1.0, abs(dg["best_lagr"])),
                       polish=dg["k"])
        rec.append(row)
        return orig(self, slot, node, st, obj, pobj, iters, inc)

    B.BranchAndBound._finish = finish
    knobs = dict(node_bound_res=float(os.environ.get("NODE_BOUND_RES", "1e-3")),
                 max_iters=int(os.environ.get("MAX_ITERS", "4096")),
                 node_max_iters=int(os.environ.get("NODE_MAX_ITERS", "0")) or None)
    print("knobs", knobs)
    bb = B.BranchAndBound(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=32,
                          tol=1e-6, time_limit=secs, upper_bound=ub * (1 + 1e-6) + 1e-6,
                          check_every=12, root_max_iters=400000, **knobs)
    t0 = time.time()
    if os.environ.get("PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        res = bb.solve()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)
    else:
        res = bb.solve()
    print(f"{N}x{F}: {time.time() - t0:.1f}s status {res.status} lps {res.lps} certified {res.certified} "
          f"drained {res.drained} inc {res.objective} bound {res.bound}")
    print("by kind:", res.lp_status_kind)
    print("timing:", {k: round(v, 2) for k, v in res.timing.items()}, "advance calls", res.advance_calls,
          "LPs in flight (mean)", round(res.inflight_sum / max(1, res.advance_calls), 1))
    for kind in ("node", "leaf", "retry"):
        rk = [r for r in rec if r["kind"] == kind]
        if not rk:
            continue
        it = np.array([r["iters"] for r in rk])
        print(f"  {kind}: {len(rk)} LPs, iterations mean {it.mean():.0f} p50 {np.median(it):.0f}, "
              f"depth mean {np.mean([r['depth'] for r in rk]):.1f}, fixings mean {np.mean([r['nfix'] for r in rk]):.0f}")
        lim = [r for r in rk if r["st"] in (LP_ITERATION_LIMIT, LP_BOUND)]
        if lim:
            pres = np.array([r["pres"] for r in lim])
            gap = np.array([r["gap"] for r in lim])
            print(f"    limit/bound {len(lim)}: pres p10/50/90 {np.percentile(pres, [10, 50, 90])}, gap p10/50/90 "
                  f"{np.percentile(gap, [10, 50, 90])}; gap<=1e-6: {(gap <= 1e-6).sum()}, pres<=1e-6: "
                  f"{(pres <= 1e-6).sum()}, both-off: {((gap > 1e-6) & (pres > 1e-6)).sum()}")
    m.close()


if __name__ == "__main__":
    main()
