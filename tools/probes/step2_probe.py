#!/usr/bin/env python3
"""Dev probe (GPU box): convergence of step-2 node LPs that do not certify.  Each LP is solved cold at
growing iteration budgets; per budget the certificate's two sides (the repaired point's objective pobj
and the bound lagr), the violation and the primal weight are printed against HiGHS, so the side that
lags is visible.

  python3 tools/step2_probe.py syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization:1   (tests/golden/golden.json)
  python3 tools/step2_probe.py scale:syn64x32_MDU_s2create                     (tests/golden/scale.json)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def case(arg):
    """(data, variant, step, kw, [(lb, ub, ref)] with the root first) of a golden / scale case."""
    if arg.startswith("scale:"):
        from scale_util import case_model_args, scale_cases
        c = scale_cases()[arg[6:]]
        data, variant, step, kw = case_model_args(c)
        return data, variant, step, kw, c["root"]["lp_objective"], [
            (nd["fix_idx"], nd["fix_val"], nd["lp_objective"]) for nd in c["nodes"]], True
    from gpu_cases import G, build_args
    name, k = arg.split(":")
    data, variant, step, kw = build_args(name, int(k))
    rec = G[name]["models"][int(k)]
    return data, variant, step, kw, rec["lp_objective"], rec.get("node_lps", []), False


def main():
    from core.engine.lp import LPModel
    budgets = [int(b) for b in os.environ.get("BUDGETS", "1000,4000,16000,64000,200000").split(",")]
    ce = int(os.environ.get("CHECK_EVERY", "64"))
    max_nodes = int(os.environ.get("MAX_NODES", "8"))
    for arg in sys.argv[1:]:
        data, variant, step, kw, rootref, nodes, scale = case(arg)
        N, F = len(data.nodes), len(data.functions)
        nodes = nodes[:max_nodes]
        B = 1 + len(nodes)
        m = LPModel(data, variant, step=step, max_batch=B, **kw)
        lb = np.full((B, m.n_int), -np.inf)
        ub = np.full((B, m.n_int), np.inf)
        refs = [rootref]
        nx = N * N * F
        for b, nd in enumerate(nodes):
            if scale:
                idx, val, ref = nd
                lb[b + 1, idx] = val
                ub[b + 1, idx] = val
            else:
                for i, v in zip(nd["fix_idx"], nd["fix_val"]):
                    lb[b + 1, i - nx] = ub[b + 1, i - nx] = v
                ref = nd["lp_objective"]
            refs.append(ref)
        print(f"== {arg} (step {step}, {variant}, {N}x{F})", flush=True)
        for it in budgets:
            res = m.solve(np.arange(B), lb, ub, tol=5e-7, max_iters=it, check_every=ce)
            for b in range(B):
                if refs[b] is None:
                    continue
                dg = m.diag(b)
                r = refs[b]
                print(f"  budget {it:7d} node {b}: st {res['status'][b]} it {res['iters'][b]:7d} "
                      f"pobj-ref {dg['pobj'] - r:+.3e} ref-bestL {r - dg['best_lagr']:+.3e} res {dg['pres']:.2e} "
                      f"omega {dg['omega']:.3g} ref {r:.9g}", flush=True)
        m.close()


if __name__ == "__main__":
    main()
