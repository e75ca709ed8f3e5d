#!/usr/bin/env python3
"""Dev probe (GPU box): primal leaves from the facility relaxation's root LP.  The root of the
bound model is solved to a converged bound, its flows / c / n are rounded by the B&B's modes and by node-first
variants (open the nodes with n >= t, then every flow-carrying placement there that memory allows), and every
leaf is solved on the reference model: status and objective per strategy.

  python3 tools/leaf_probe.py 128x64 256x128
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def node_first(F, N, flow, c, n, fmem, nmem, t):
    """open the nodes with n >= t; per open node, placements by decreasing flow while memory allows; every
    function without a placement gets its largest-flow open node with room (else the next node by n)"""
    openj = n >= t
    C = np.zeros((F, N))
    used = np.zeros(N)
    order = np.argsort(-flow, axis=None, kind="stable")
    for k in order:
        f, j = divmod(int(k), N)
        if not openj[j] or flow[f, j] <= 1e-4:
            continue
        if used[j] + fmem[f] <= nmem[j] + 1e-9:
            C[f, j] = 1.0
            used[j] += fmem[f]
    for f in np.flatnonzero(C.sum(axis=1) < 1):
        cand = sorted(range(N), key=lambda j: (-int(openj[j]), -flow[f, j], -n[j]))
        for j in cand:
            if used[j] + fmem[f] <= nmem[j] + 1e-9:
                C[f, j] = 1.0
                used[j] += fmem[f]
                break
        else:
            return None
    nn = (C.sum(axis=0) > 0).astype(float)
    return np.concatenate([np.arange(F * N + N)]), np.concatenate([C.ravel(), nn])


def main():
    from core.engine.bnb import BranchAndBound, _Node, NODE
    from core.engine.lp import LPModel, LP_OPTIMAL, RELAX_FACILITY
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    for size in sys.argv[1:]:
        N, F = (int(t) for t in size.split("x"))
        p = synthetic_payload(N, F, seed=0)
        data = data_to_solver_input(p, with_db=False)
        fm = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=1, relaxation=RELAX_FACILITY)
        t0 = time.perf_counter()
        r = fm.solve([0], tol=1e-6, gap_tol=1e-4, bound_res=1e-2, max_iters=400000, check_every=64)
        flow = fm.flows([0])[0].astype(np.float64)
        z, _ = fm.solution(0, dense_x=False)
        fm.close()
        c, n = z[:F * N], z[F * N:]
        print(f"{size}: fac root status {r['status'][0]} bound {r['obj'][0]:.6g} iters {r['iters'][0]} "
              f"{time.perf_counter() - t0:.1f}s; sum n {n.sum():.2f}, n>0.5 {(n > 0.5).sum()}, n>0.01 {(n > 0.01).sum()}",
              flush=True)
        fmem = np.asarray(data.function_memory_matrix, float)
        nmem = np.asarray(data.node_memory_matrix, float)
        leaves = []

        class _L:
            pass
        lpstub = _L()
        lpstub.N, lpstub.F, lpstub.max_batch, lpstub.n_int = N, F, 4, F * N + N
        lpstub.layout = lambda: {"c": (0, F * N), "n": (F * N, F * N + N)}
        bb = BranchAndBound(lpstub, data.workload_matrix, fmem, nmem)
        root = _Node(0, np.zeros(0, np.int64), np.zeros(0), NODE, None, 0)
        for by_flow, mf in bb.round_modes:
            lf = bb._round(root, flow.astype(np.float32), c, by_flow, mf)
            leaves.append((f"round by_flow={by_flow} min_flow={mf}", lf))
        for t in (0.5, 0.2, 0.1, 0.05, 0.02, 0.01, 1e-3):
            leaves.append((f"node-first n>={t}", node_first(F, N, flow.reshape(F, N), c, n, fmem, nmem, t)))
        good = [(nm, lf) for nm, lf in leaves if lf is not None]
        for nm, lf in leaves:
            if lf is None:
                print(f"   {nm}: no leaf", flush=True)
        m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=len(good) + 1)
        rr = m.solve([len(good)], tol=1e-6, max_iters=400000)
        lb = np.full((len(good), m.n_int), -np.inf)
        ub = np.full((len(good), m.n_int), np.inf)
        for b, (nm, (idx, val)) in enumerate(good):
            lb[b, idx] = ub[b, idx] = val
            m.copy_state(len(good), b)
        t0 = time.perf_counter()
        res = m.solve(np.arange(len(good)), lb, ub, tol=1e-6, max_iters=40000, check_every=12, warm_start=True)
        for b, (nm, (idx, val)) in enumerate(good):
            cc = val[:F * N]
            print(f"   {nm}: open c {int(cc.sum())} nodes {int(val[F * N:].sum())}: leaf status {res['status'][b]} "
                  f"obj {res['primal_obj'][b]:.6g} bound {res['obj'][b]:.6g} iters {res['iters'][b]}", flush=True)
        print(f"   (ref root {rr['iters'][0]} iterations; leaves {time.perf_counter() - t0:.1f}s)", flush=True)
        m.close()


if __name__ == "__main__":
    main()
