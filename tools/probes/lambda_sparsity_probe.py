#!/usr/bin/env python3
"""Dev probe (GPU box): how sparse the facility relaxation's x <= c dual rows (nonzeros per row) and the routing
anchors (nonzeros as held, 17 = dense) are (nep_debug_sparse_rows) — its root LP after a few thousand iterations and
warm children after a branching node's budget — and the seconds per LP-iteration (DESIGN.md §7 "Sparse facility
duals": a (j, value)-pair storage of the dual rows was built on these counts, measured and removed).

  python3 tools/probe.py lambda_sparsity_probe 512x256 [root_iters] [child_iters]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402


def hist(c):
    c = np.asarray(c)
    return {"rows": int(c.size), "empty": int((c == 0).sum()), "le4": int(((c > 0) & (c <= 4)).sum()),
            "le16": int(((c > 4) & (c <= 16)).sum()), "dense": int((c > 16).sum()),
            "mean_sparse": float(c[c <= 16].mean()) if (c <= 16).any() else None}


def main():
    import torch
    torch.cuda.set_device(0)
    from core.engine.lp import LPModel, RELAX_FACILITY
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    size = sys.argv[1] if len(sys.argv) > 1 else "512x256"
    root_iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    child_iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    N, F = (int(t) for t in size.split("x"))
    p = synthetic_payload(N, F, seed=0)
    data = data_to_solver_input(p, with_db=False)
    B = 8
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=B + 1,
                relaxation=RELAX_FACILITY)
    t = time.perf_counter()
    r = m.solve([B], tol=1e-6, max_iters=root_iters, check_every=64)
    dt = time.perf_counter() - t
    a, lam = m.sparse_rows(B)
    print(f"{size} facility root: status {int(r['status'][0])} iters {int(r['iters'][0])} {dt:.2f}s "
          f"({dt / max(1, int(r['iters'][0])) * 1e6:.1f} us/iter)", flush=True)
    print("  lambda", hist(lam), flush=True)
    print("  anchor", hist(a), flush=True)
    rng = np.random.default_rng(1)
    lb = np.full((B, m.n_int), -np.inf)
    ub = np.full((B, m.n_int), np.inf)
    for b in range(B):
        j = int(rng.integers(N))
        lb[b, F * N + j] = ub[b, F * N + j] = float(b % 2)
        m.copy_state(B, b)
    t = time.perf_counter()
    rr = m.solve(np.arange(B), lb, ub, tol=1e-6, max_iters=child_iters, warm_start=True, check_every=12)
    dt = time.perf_counter() - t
    its = int(np.max(rr["iters"]))
    print(f"  {B} warm children: statuses {rr['status'].tolist()} iters {rr['iters'].tolist()} {dt:.2f}s "
          f"({dt / max(1, its) * 1e6:.1f} us per batched iteration)", flush=True)
    lams = np.concatenate([m.sparse_rows(b)[1] for b in range(B)])
    print("  children lambda", hist(lams), flush=True)
    m.close()


if __name__ == "__main__":
    main()
