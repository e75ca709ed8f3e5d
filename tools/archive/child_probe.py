#!/usr/bin/env python3
"""Dev probe (GPU box): iteration distribution of bench.py's warm-started child LPs.

Solves the first `--probe-n` nodes of rank 0's node stream (same seeds as bench.NodeStream) in
batches of `--batch`, warm-started from the root, and prints per node: status, iterations, the
fixings (f, j, value) with the root's c value there, and for unfinished nodes the final residual
and gap."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    n_probe = 48
    if "--probe-n" in argv:
        i = argv.index("--probe-n")
        n_probe = int(argv[i + 1])
        del argv[i:i + 2]
    a = bench.parse(argv)
    import torch
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    B = a.batch
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=B + 1)
    t = time.perf_counter()
    rr = m.solve([B], tol=a.tol, max_iters=a.root_max_iters, check_every=a.check_every)
    print(f"root st={rr['status'][0]} it={rr['iters'][0]} obj={rr['obj'][0]:.10g} {time.perf_counter() - t:.2f}s",
          flush=True)
    c_root = m.solution(B, dense_x=False)[0][: a.functions * a.nodes]
    for b0 in range(0, n_probe, B):
        nb = min(B, n_probe - b0)
        lbs, ubs = [], []
        for k in range(b0, b0 + nb):
            seed = (a.seed * 1000003 + 0) * 7919 + k
            lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, seed)
            lbs.append(lb[0])
            ubs.append(ub[0])
        for s in range(nb):
            if not a.cold:
                m.copy_state(B, s)
        t = time.perf_counter()
        r = m.solve(np.arange(nb), np.array(lbs), np.array(ubs), tol=a.tol, max_iters=a.max_iters,
                    check_every=a.check_every, warm_start=not a.cold)
        dt = time.perf_counter() - t
        print(f"batch {b0 // B}: {dt:.2f}s", flush=True)
        for s in range(nb):
            fx = np.nonzero(np.isfinite(lbs[s]))[0]
            desc = ", ".join(f"c[{i // a.nodes},{i % a.nodes}]={int(lbs[s][i])} (root {c_root[i]:.3g})" for i in fx)
            line = f"  node {b0 + s}: st={r['status'][s]} it={r['iters'][s]} obj={r['obj'][s]:.10g} | {desc}"
            if r["status"][s] != 0 and r["status"][s] != 2:
                dg = m.diag(s)
                line += f" | pres={dg['pres']:.3g} gap={dg['gap']:.3g} omega={dg['omega']:.3g}"
            print(line, flush=True)
    m.close()


if __name__ == "__main__":
    main()
