#!/usr/bin/env python3
"""Dev probe (GPU box): how the bench's 512x256 root LP and the node LPs warm-started from it depend on the
step size.  For each eta scale (NEP_ETA_SCALE, read by nep_model_create): the cold root (iterations, seconds,
final primal weight), then 32 root children (2 random c[f, j] fixed each, seeded) warm-started from it —
their iteration distribution and certified count at a 20000-iteration budget.

  python3 tools/root_chaos_probe.py 1 0.999999999999 1.000000001 0.999
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]


def main():
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F = int(os.environ.get("ROOT_N", 512)), int(os.environ.get("ROOT_F", 256))
    seed = int(os.environ.get("ROOT_SEED", 0))
    B = 32
    data = data_to_solver_input(synthetic_payload(N, F, seed=seed), with_db=False)
    rng = np.random.default_rng(7)
    fix = [(rng.choice(F * N, 2, replace=False), rng.integers(0, 2, 2).astype(float)) for _ in range(B)]
    for arg in sys.argv[1:] or ["1"]:
        os.environ["NEP_ETA_SCALE"] = arg
        m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=B + 1)
        t = time.perf_counter()
        r = m.solve([B], tol=1e-6, max_iters=400000, check_every=64)
        dt = time.perf_counter() - t
        dg = m.diag(B)
        lb = np.full((B, m.n_int), -np.inf)
        ub = np.full((B, m.n_int), np.inf)
        for b, (idx, val) in enumerate(fix):
            lb[b, idx] = val
            ub[b, idx] = val
        for b in range(B):
            m.copy_state(B, b)
        t2 = time.perf_counter()
        c = m.solve(list(range(B)), lb, ub, tol=1e-6, max_iters=20000, check_every=64, warm_start=True)
        dt2 = time.perf_counter() - t2
        it = c["iters"]
        print(f"scale {arg:>16s} eta {m.info.step_size:.15g} root st {int(r['status'][0])} iters {int(r['iters'][0])} "
              f"{dt:.2f}s omega {dg['omega']:.4g} | children mean {it.mean():.0f} p50 {np.median(it):.0f} "
              f"p90 {np.percentile(it, 90):.0f} certified {(c['status'] == 0).sum()}/{B} {dt2:.2f}s", flush=True)
        m.close()


if __name__ == "__main__":
    main()
