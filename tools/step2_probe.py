#!/usr/bin/env python3
"""Dev probe (GPU box): convergence of step-2 node LPs that do not certify.  Each golden LP is solved
cold at growing iteration budgets; per budget the certificate's two sides (the repaired point's
objective pobj and the bound lagr), the violation and the primal weight are printed against HiGHS,
so the side that lags is visible.

  python3 tools/step2_probe.py syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization:1
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    from core.engine.lp import LPModel
    from gpu_cases import G, build_args, fixing_bounds
    budgets = [int(b) for b in os.environ.get("BUDGETS", "1000,4000,16000,64000,200000").split(",")]
    ce = int(os.environ.get("CHECK_EVERY", "64"))
    for nk in sys.argv[1:]:
        name, k = nk.split(":")
        k = int(k)
        data, variant, step, kw = build_args(name, k)
        rec = G[name]["models"][k]
        N, F = len(data.nodes), len(data.functions)
        m = LPModel(data, variant, step=step, max_batch=1 + len(rec.get("node_lps", [])), **kw)
        nodes = fixing_bounds(name, k, m.n_int, N * N * F)
        B = 1 + len(nodes)
        lb = np.full((B, m.n_int), -np.inf)
        ub = np.full((B, m.n_int), np.inf)
        for b, (l, u, _) in enumerate(nodes):
            lb[b + 1], ub[b + 1] = l, u
        refs = [rec["lp_objective"]] + [r for _, _, r in nodes]
        print(f"== {name} model {k} (step {step}, {variant}, {N}x{F})", flush=True)
        for it in budgets:
            res = m.solve(np.arange(B), lb, ub, tol=5e-7, max_iters=it, check_every=ce)
            for b in range(B):
                if refs[b] is None:
                    continue
                dg = m.diag(b)
                r = refs[b]
                print(f"  budget {it:7d} node {b}: st {res['status'][b]} it {res['iters'][b]:7d} "
                      f"pobj-ref {dg['pobj'] - r:+.3e} ref-lagr {r - dg['lagr']:+.3e} res {dg['pres']:.2e} "
                      f"omega {dg['omega']:.3g} ref {r:.9g}", flush=True)
        m.close()


if __name__ == "__main__":
    main()
