#!/usr/bin/env python3
"""Dev probe (GPU box): wall time per PDHG iteration of small single LPs (payload.json step 1 and
step 2, synthetic 64x32 / 128x64 roots) — the launch-latency-bound regime."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]


def main():
    import torch
    from core.engine.lp import LPModel, STEP1
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    from golden_util import payload
    torch.cuda.set_device(0)
    cases = [("payload", payload("payload"), 20000)]
    for n, f in ((64, 32), (128, 64)):
        cases.append((f"{n}x{f}", synthetic_payload(n, f, seed=0), 200000))
    for name, p, iters in cases:
        d = data_to_solver_input(p, with_db=False)
        alpha = p["solver"]["args"].get("alpha", 0.5)
        m = LPModel(d, "MinDelayAndUtilization", step=STEP1, alpha=alpha, max_batch=1)
        m.solve([0], tol=1e-6, max_iters=64)   # warm-up (module load, first launches)
        t = time.perf_counter()
        r = m.solve([0], tol=1e-6, max_iters=iters)
        dt = time.perf_counter() - t
        it = int(r["iters"][0])
        print(f"{name}: status {r['status'][0]} obj {r['obj'][0]:.10g} iters {it} {dt:.3f}s "
              f"= {1e6 * dt / max(1, it):.1f} us/iteration", flush=True)
        m.close()


if __name__ == "__main__":
    main()
