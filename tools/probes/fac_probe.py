#!/usr/bin/env python3
"""Dev probe (GPU box): the facility relaxation's root LP (NEP_RELAX_FACILITY) against the
reference relaxation's at growing sizes — status, iterations, seconds, value — and a few warm children.

  python3 tools/fac_probe.py 64x32 256x128 512x256
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    from core.engine.lp import LPModel, RELAX_FACILITY, RELAX_REFERENCE
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    for size in sys.argv[1:]:
        N, F = (int(t) for t in size.split("x"))
        p = synthetic_payload(N, F, seed=0)
        data = data_to_solver_input(p, with_db=False)
        for rel in (RELAX_FACILITY, RELAX_REFERENCE):
            m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=5, relaxation=rel)
            t0 = time.perf_counter()
            r = m.solve([4], tol=1e-6, max_iters=400000, check_every=64)
            t1 = time.perf_counter()
            d = m.diag(4)
            print(f"{size} relax {rel}: root status {r['status'][0]} obj {r['obj'][0]:.9g} pobj {r['primal_obj'][0]:.9g} "
                  f"iters {r['iters'][0]} {t1 - t0:.2f}s res {d['pres']:.2e}", flush=True)
            rng = np.random.default_rng(1)
            lb = np.full((4, m.n_int), -np.inf)
            ub = np.full((4, m.n_int), np.inf)
            for b in range(4):
                j = int(rng.integers(N))
                lb[b, F * N + j] = ub[b, F * N + j] = float(b % 2)
                m.copy_state(4, b)
            t0 = time.perf_counter()
            c = m.solve(np.arange(4), lb, ub, tol=1e-6, max_iters=100000, check_every=12, warm_start=True)
            print(f"   children (n fixings): status {c['status'].tolist()} iters {c['iters'].tolist()} "
                  f"obj {[round(float(o), 9) for o in c['obj']]} {time.perf_counter() - t0:.2f}s", flush=True)
            m.close()


if __name__ == "__main__":
    main()
