#!/usr/bin/env python3
"""Dev probe (GPU box): bench.py's node stream with a log line per advance() call — wall time of the
call, iterating slots before/after, the slots that finished with their status and iteration
count — to see where a streaming step's time goes (slot occupancy, host refill, LP iterations)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import bench  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:])
    import torch
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=a.batch + 1)
    t = time.perf_counter()
    rr = m.solve([a.batch], tol=a.tol, max_iters=a.root_max_iters, check_every=a.check_every)
    print(f"root st={rr['status'][0]} it={rr['iters'][0]} {time.perf_counter() - t:.2f}s", flush=True)
    s = bench.NodeStream(m, a.batch, a, 0)
    t = time.perf_counter()
    s.fill()
    print(f"fill {time.perf_counter() - t:.3f}s active={m.active()}", flush=True)
    m.reset_stats()
    t0 = time.perf_counter()
    for call in range(40):
        t = time.perf_counter()
        n0 = m.active()
        r = m.advance(1)
        ta = time.perf_counter() - t
        t = time.perf_counter()
        for sl in r["slots"]:
            s._start(int(sl))
        tr = time.perf_counter() - t
        print(f"call {call}: active {n0} advance {ta * 1e3:.1f} ms refill {tr * 1e3:.1f} ms done "
              f"{list(zip(r['status'].tolist(), r['iters'].tolist()))}", flush=True)
    st = m.stats()
    print(f"total {time.perf_counter() - t0:.2f}s stats {st}", flush=True)
    m.close()


if __name__ == "__main__":
    main()
