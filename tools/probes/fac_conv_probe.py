#!/usr/bin/env python3
"""Dev probe (GPU box): convergence trace of facility-relaxation LPs that end at the iteration limit — the
test_gpu_fac.py cases, each LP continued in chunks (warm, from its own state), printing the certificate's
primal objective, the Lagrangian bound, the relative residual, the gap and the primal weight per chunk.

  python3 tools/fac_conv_probe.py 32x16:MinUtilization 64x32:MinDelayAndUtilization   [CHUNK=20000 CHUNKS=8]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
from test_gpu_fac import _fixings  # noqa: E402


def main():
    from core.engine.lp import LPModel, RELAX_FACILITY
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    chunk, chunks = int(os.environ.get("CHUNK", "20000")), int(os.environ.get("CHUNKS", "8"))
    for arg in sys.argv[1:]:
        size, variant = arg.split(":")
        N, F = (int(t) for t in size.split("x"))
        p = synthetic_payload(N, F, seed=0)
        data = data_to_solver_input(p, with_db=False)
        fix = _fixings(F, N, np.random.default_rng(N + F), 4)
        B = len(fix)
        m = LPModel(data, variant, step=1, alpha=p["solver"]["args"]["alpha"], max_batch=B + 1,
                    relaxation=RELAX_FACILITY)
        lb = np.full((B + 1, m.n_int), -np.inf)
        ub = np.full((B + 1, m.n_int), np.inf)
        for b, (idx, val) in enumerate(fix):
            lb[b, idx] = ub[b, idx] = val
        for b in [B] + list(range(B)):
            for c in range(chunks):
                r = m.solve([b], lb[b:b + 1], ub[b:b + 1], tol=5e-7, max_iters=chunk, warm_start=c > 0)
                d = m.diag(b)
                print(f"{arg} LP {b} chunk {c}: st {r['status'][0]} it {r['iters'][0]} obj {r['obj'][0]:.10g} "
                      f"pobj {d['pobj']:.10g} best_lagr {d['best_lagr']:.10g} pres {d['pres']:.2e} gap {d['gap']:.2e} "
                      f"omega {d['omega']:.3g} k {d['k']:.0f}", flush=True)
                if r["status"][0] == 0:
                    break
            if b == B:
                for k in range(B):
                    m.copy_state(B, k)
        m.close()


if __name__ == "__main__":
    main()
