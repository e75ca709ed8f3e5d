#!/usr/bin/env python3
"""Dev probe (GPU box): support sizes of the routing rows' T outputs (points on the simplexes).

The Halpern anchor is always such a point (it is set from the iterate right after a plain
certificate iteration), so a row's support size bounds what a compressed anchor must hold.  The
iterate itself is a Halpern combination of T outputs since the last restart: the union of the
supports of consecutive snapshots estimates its support.

Reports, for the bench's 512x256 root LP (cold solves cut at several iteration counts; each run
is deterministic, so the cuts are snapshots of one trajectory) and for bench children that reach
the node-LP iteration limit, the distribution of per-row nonzero counts."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def describe(tag, nnz, N):
    q = np.percentile(nnz, [50, 90, 99, 100])
    frac = {k: float(np.mean(nnz <= k)) for k in (1, 2, 4, 8, 16, 32, 64)}
    print(f"{tag}: rows {nnz.size} nnz p50/p90/p99/max {q.tolist()} mean {nnz.mean():.2f} (N={N}) "
          f"frac<=k {frac}", flush=True)


def main():
    a = bench.parse(sys.argv[1:])
    import torch
    from core.engine.lp import LPModel, LP_OPTIMAL
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    alpha = p["solver"]["args"]["alpha"]
    B = a.batch
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=B + 1)
    root = B
    snaps = {}
    for k in (256, 1024, 4096, 4096 + 64, 4096 + 128, 4096 + 256, 16384):
        t = time.time()
        r = m.solve([root], tol=a.tol, max_iters=k, check_every=a.root_check_every)
        xb, _, _ = m.rows(root)
        snaps[k] = xb != 0
        describe(f"root cut {k} (st {r['status'][0]}, {time.time() - t:.2f}s)", snaps[k].sum(1), m.N)
    u = snaps[4096] | snaps[4096 + 64] | snaps[4096 + 128] | snaps[4096 + 256]
    describe("root union of cuts 4096..4352", u.sum(1), m.N)
    r = m.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every)
    xb, _, _ = m.rows(root)
    describe(f"root final (st {r['status'][0]}, it {r['iters'][0]})", (xb != 0).sum(1), m.N)
    # children: the bench's node stream, first 2*B nodes
    counter = 0
    lbs, ubs, slots = [], [], list(range(B))
    for s in slots:
        lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, (a.seed * 1000003) * 7919 + counter)
        counter += 1
        lbs.append(lb[0])
        ubs.append(ub[0])
        m.copy_state(root, s)
    m.submit(slots, np.array(lbs), np.array(ubs), tol=a.tol, max_iters=a.max_iters, check_every=a.check_every,
             warm_start=True)
    allnz = []
    while m.active() > 0:
        rr = m.advance(1)
        for i, s in enumerate(rr["slots"].tolist()):
            xb, _, _ = m.rows(s)
            nz = (xb != 0).sum(1)
            allnz.append(nz)
            if int(rr["status"][i]) != LP_OPTIMAL:
                describe(f"child slot {s} status {rr['status'][i]} it {rr['iters'][i]}", nz, m.N)
    describe("all children (final T outputs)", np.concatenate(allnz), m.N)
    m.close()


if __name__ == "__main__":
    main()
