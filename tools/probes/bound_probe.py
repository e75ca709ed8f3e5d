#!/usr/bin/env python3
"""Dev probe (GPU box): why the step-1 search's bound stalls (round-5 VERDICT #1).  Runs the product's two-model
search (NeptuneStepBase.branch_and_bound: facility-relaxation branching nodes, reference-model leaves) on the
Python loop (NEP_BNB_PYTHON=1: per-LP hooks) and records, per finished branching-node LP: its parent's bound,
its own LP bound, status, iterations, depth, the branching variable that created it (n or c, and its value), and
the global bound (min over open nodes) over time.  Prints a JSON summary: how often a child's LP raises the bound
over its parent's, by status (bound-converged / iteration limit) and by branching kind.

  python3 tools/bound_probe.py N F seconds [seed] [--node-iters K] [--bound-gap G] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]
os.environ["NEP_BNB_PYTHON"] = "1"

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("N", type=int)
    ap.add_argument("F", type=int)
    ap.add_argument("seconds", type=float)
    ap.add_argument("seed", type=int, nargs="?", default=0)
    ap.add_argument("--node-iters", type=int, default=0, help="branching-node LP budget (0: the product's)")
    ap.add_argument("--bound-gap", type=float, default=0.0, help="bound model gap_tol (0: the product's 1e-4)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from core.engine import bnb as B
    from core.engine.lp import LPModel, LP_BOUND, LP_ITERATION_LIMIT, LP_OPTIMAL
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    p = synthetic_payload(a.N, a.F, seed=a.seed)
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6, lp_max_iters=4096)
    st1.load_data(data)
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    bm = st1.bound_model(data, 33)
    FN = a.F * a.N
    rec, glob = [], []
    orig = B.BranchAndBound._finish
    t0 = [None]

    def finish(self, eng, slot, node, st, obj, pobj, iters, inc, pre=None):
        if t0[0] is None:
            t0[0] = time.time()
        if node.kind == B.NODE and node.depth > 0 and eng is self.B:
            v = int(node.idx[-1]) if len(node.idx) else -1
            rec.append({"depth": node.depth, "parent_bound": node.bound, "lp": obj, "st": int(st), "iters": int(iters),
                        "var": "n" if v >= FN else "c", "val": float(node.val[-1]) if len(node.val) else None,
                        "inc": inc})
        out = orig(self, eng, slot, node, st, obj, pobj, iters, inc, pre)
        if len(rec) % 50 == 0 and self.heap:
            glob.append((time.time() - t0[0], min(h[0] for h in self.heap), out))
        return out

    B.BranchAndBound._finish = finish
    ov = dict(time_limit=a.seconds, root_max_iters=400000)
    if a.node_iters:
        ov["node_max_iters"] = a.node_iters
    if a.bound_gap:
        ov["bound_gap"] = a.bound_gap
    bb = st1.branch_and_bound(m, bm, **ov)
    res = bb.solve()
    m.close()
    bm.close()
    d = np.array([r["lp"] - r["parent_bound"] for r in rec]) if rec else np.zeros(0)
    sts = np.array([r["st"] for r in rec]) if rec else np.zeros(0)
    out = {"instance": f"{a.N}x{a.F}_s{a.seed}", "seconds": a.seconds, "status": res.status, "incumbent": res.objective,
           "bound": res.bound, "nodes": res.nodes, "lps": res.lps, "node_lps": len(rec),
           "raised_share": float((d > 1e-9).mean()) if d.size else None,
           "raise_p50_p90_max": [float(x) for x in np.percentile(d, [50, 90, 100])] if d.size else None,
           "by_status": {}, "by_var": {}, "global_bound_trace": glob[:: max(1, len(glob) // 40)]}
    for name, code in (("bound", LP_BOUND), ("limit", LP_ITERATION_LIMIT), ("certified", LP_OPTIMAL)):
        sel = sts == code
        if sel.any():
            out["by_status"][name] = {"lps": int(sel.sum()), "raised_share": float((d[sel] > 1e-9).mean()),
                                      "mean_iters": float(np.mean([r["iters"] for r, s in zip(rec, sel) if s]))}
    for var in ("n", "c"):
        for val in (0.0, 1.0):
            sel = np.array([r["var"] == var and r["val"] == val for r in rec])
            if sel.size and sel.any():
                out["by_var"][f"{var}={int(val)}"] = {"lps": int(sel.sum()), "raised_share": float((d[sel] > 1e-9).mean()),
                                                      "raise_mean": float(d[sel].mean())}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"summary": out, "records": rec}, fh)


if __name__ == "__main__":
    main()
