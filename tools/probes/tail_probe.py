#!/usr/bin/env python3
"""Dev probe (GPU box): which of bench.py's node LPs reach the node-LP iteration limit, and why.

Streams the bench's first `--probe-nodes` children (same seeds as bench.py), records the ones that
stop uncertified, prints their final diagnostics (nep_lp_get_diag), then re-solves them with a
large iteration budget and reports whether they certify, how fast, and where their Lagrangian
bound ends against the a-priori objective bound the product B&B uses as cutoff."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def family_residuals(m, slot, data, dbg):
    """max normalised violation per dualised row family at the slot's last certificate iteration
    (row activities kz of the T output; rownorm from nep_debug_build)."""
    import ctypes
    from core.engine.lp import _ptr
    n_dual = dbg["n_dual"]
    y = np.zeros(n_dual)
    kz = np.zeros(n_dual)
    m._lib.nep_debug_state(m._h, int(slot), _ptr(y), _ptr(kz), None, None, None)
    F, N = m.F, m.N
    FN = F * N
    o = {"C1": (0, FN), "C2": (FN, 2 * FN), "C3": (2 * FN, 2 * FN + N), "C5": (2 * FN + N, 2 * FN + 2 * N),
         "C6": (2 * FN + 2 * N, 2 * FN + 3 * N), "C7": (2 * FN + 3 * N, 2 * FN + 4 * N)}
    lo = np.full(n_dual, -np.inf)
    hi = np.full(n_dual, np.inf)
    hi[0:FN] = 0.0
    lo[FN:2 * FN] = -1e-6
    hi[2 * FN:2 * FN + N] = np.asarray(data.node_memory_matrix, float)
    hi[2 * FN + N:2 * FN + 2 * N] = np.asarray(data.node_cores_matrix, float)
    hi[2 * FN + 2 * N:2 * FN + 3 * N] = 0.0
    lo[2 * FN + 3 * N:2 * FN + 4 * N] = -1e-6
    v = np.maximum(np.maximum(lo - kz, kz - hi), 0.0) / dbg["rownorm"]
    out = {}
    for k, (a, b) in o.items():
        i = int(np.argmax(v[a:b]))
        out[k] = (float(v[a + i]), a + i - o[k][0], float(y[a + i]))
    return out


def main():
    argv = sys.argv[1:]
    n_probe = 160
    if "--probe-nodes" in argv:
        i = argv.index("--probe-nodes")
        n_probe = int(argv[i + 1])
        del argv[i:i + 2]
    a = bench.parse(argv)
    import torch
    from core.engine.lp import LPModel, LP_OPTIMAL
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.engine.lp import debug_build
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    alpha = p["solver"]["args"]["alpha"]
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=alpha)
    st1.load_data(d)
    ub0 = st1.upper_bound()
    dbg = debug_build(d, "MinDelayAndUtilization", alpha=alpha)
    B = a.batch
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=B + 1)
    root = B
    t = time.time()
    rr = m.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every)
    print(f"root st={rr['status'][0]} it={rr['iters'][0]} obj={rr['obj'][0]:.10g} ({time.time() - t:.2f}s) "
          f"a-priori ub={ub0:.6g}", flush=True)
    seeds = {}
    res = {}
    counter = 0

    def refill(free):
        nonlocal counter
        take = [s for s in free][: max(0, n_probe - counter)]
        if not take:
            return
        lbs, ubs = [], []
        for s in take:
            seed = (a.seed * 1000003) * 7919 + counter
            seeds[s] = (counter, seed)
            counter += 1
            lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, seed)
            lbs.append(lb[0])
            ubs.append(ub[0])
            m.copy_state(root, s)
        st = m.submit(take, np.array(lbs), np.array(ubs), tol=a.tol, max_iters=a.max_iters,
                      check_every=a.check_every, warm_start=True)
        for s, c in zip(take, st):
            if int(c) == 2:
                res[seeds[s][0]] = (2, 0, None)
                refill([s])

    refill(range(B))
    while m.active() > 0:
        r = m.advance(1)
        for i, s in enumerate(r["slots"].tolist()):
            k, seed = seeds[s]
            dg = m.diag(s) if int(r["status"][i]) != LP_OPTIMAL else None
            if dg is not None:
                dg["fam"] = family_residuals(m, s, d, dbg)
            res[k] = (int(r["status"][i]), int(r["iters"][i]), dg)
        refill(r["slots"].tolist())
    its = np.array([v[1] for v in res.values()])
    hard = sorted(k for k, v in res.items() if v[0] != LP_OPTIMAL)
    print(f"{len(res)} nodes: certified {sum(v[0] == 0 for v in res.values())}, iters p50/p90/max "
          f"{np.percentile(its, [50, 90, 100]).tolist()}, total {its.sum()}, uncertified {hard}", flush=True)
    for k in hard:
        st, it, dg = res[k]
        if dg is None:
            print(f"  node {k}: status {st} (presolve)")
            continue
        print(f"  node {k}: status {st} it {it} pobj {dg['pobj']:.6g} lagr {dg['lagr']:.6g} best {dg['best_lagr']:.6g} "
              f"pres {dg['pres']:.3g} gap {dg['gap']:.3g} omega {dg['omega']:.3g} ksr {dg['k_since_restart']:.0f}",
              flush=True)
        print("      families: " + " ".join(f"{k}={v[0]:.2g}@{v[1]}(y={v[2]:.3g})" for k, v in dg["fam"].items()),
              flush=True)
    # re-solve the hard ones with a large budget
    hard = [k for k in hard if res[k][2] is not None][:B]
    if hard:
        lbs, ubs = [], []
        for b, k in enumerate(hard):
            lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, (a.seed * 1000003) * 7919 + k)
            lbs.append(lb[0])
            ubs.append(ub[0])
            m.copy_state(root, b)
        t = time.time()
        r = m.solve(np.arange(len(hard)), np.array(lbs), np.array(ubs), tol=a.tol, max_iters=60000,
                    check_every=a.check_every, warm_start=True)
        print(f"re-solve of {len(hard)} hard nodes at 60000 iterations ({time.time() - t:.1f}s):", flush=True)
        for b, k in enumerate(hard):
            dg = m.diag(b)
            fx = np.flatnonzero(np.isfinite(lbs[b]))
            print(f"  node {k}: status {r['status'][b]} it {r['iters'][b]} obj {r['obj'][b]:.8g} "
                  f"pobj {r['primal_obj'][b]:.8g} pres {dg['pres']:.3g} gap {dg['gap']:.3g} omega {dg['omega']:.3g} "
                  f"fix {[(int(i), float(lbs[b][i])) for i in fx]}", flush=True)
    m.close()


if __name__ == "__main__":
    main()
