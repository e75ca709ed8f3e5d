#!/usr/bin/env python3
"""Dev probe (GPU box): a scale.json case's node LPs warm-started from its root (tests/test_gpu_scale.py's
_solve_case) at a larger iteration limit, with and without the model reference weight — the one LP the
NEP_INLINE_REFLECT build does not certify within 200k iterations (syn64x32_MDU_s2delete node 2).

  NEPTUNE_LP_LIB=.../libneptune_lp_refl.so python3 tools/refl_node_probe.py syn64x32_MDU_s2delete
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    from core.engine.lp import LPModel
    from scale_util import case_model_args, node_bounds, scale_cases
    c = scale_cases()[sys.argv[1]]
    data, variant, step, kw = case_model_args(c)
    B = len(c["nodes"])
    for wref in (0.0, 8.0):
        m = LPModel(data, variant, step=step, max_batch=B + 1, **kw)
        rr = m.solve([B], tol=1e-6, max_iters=400000)
        if wref:
            m.set_reference_weight(wref * m.info.primal_weight0)
        lb, ub = node_bounds(c, m.n_int)
        for b in range(B):
            m.copy_state(B, b)
        res = m.solve(np.arange(B), lb, ub, tol=1e-6, max_iters=800000, warm_start=True)
        print(f"{sys.argv[1]} wref {wref}: root {int(rr['iters'][0])} st {int(rr['status'][0])}; nodes st "
              f"{res['status'].tolist()} iters {res['iters'].tolist()}", flush=True)
        m.close()


if __name__ == "__main__":
    main()
