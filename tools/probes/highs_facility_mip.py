#!/usr/bin/env python3
"""CPU probe: HiGHS (scipy milp) on the step-1 MinDelayAndUtilization FACILITY MIP of a SURVEY §8(d) instance —
the reference's rows with exact zero-workload aggregation, x <= c, c <= n, capacities scaled by n and C2's eps floor
kept (so its integral optimum is the reference MIP's) — as the yardstick for the GPU search's closing (DESIGN.md §7
"Closing the search"; profiles/r06/highs).  Prints the LP relaxation (value, sum n, fractional n) and the MIP
(objective, HiGHS dual bound, status, seconds).

  python3 tools/probe.py highs_facility_mip N F [time_limit_s]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]
from core.utils.synthetic import synthetic_payload
from core.utils import data_to_solver_input
from scipy.optimize import milp, LinearConstraint, Bounds

def build(N, F, seed=0, alpha=0.5, c2=True, extra=()):
    p = synthetic_payload(N, F, seed=seed)
    d = data_to_solver_input(p, with_db=False)
    W = np.asarray(d.workload_matrix, float); D = np.asarray(d.node_delay_matrix, float)
    cpr = np.asarray(d.core_per_req_matrix, float); cores = np.asarray(d.node_cores_matrix, float).ravel()
    fm = np.asarray(d.function_memory_matrix, float).ravel(); nm = np.asarray(d.node_memory_matrix, float).ravel()
    mwd = float((W * D.max(axis=1)[None, :]).sum())
    rows = []  # (f, i or -1, weight)
    for f in range(F):
        for i in np.flatnonzero(W[f] > 0): rows.append((f, int(i), 1.0))
        m0 = int((W[f] == 0).sum())
        if m0: rows.append((f, -1, float(m0)))
    R = len(rows)
    nx = R * N; c0 = nx; n0 = nx + F * N; nv = n0 + N
    cost = np.zeros(nv)
    for r, (f, i, w) in enumerate(rows):
        if i >= 0: cost[r * N:(r + 1) * N] = (1 - alpha) * W[f, i] * D[i] / mwd
    cost[n0:] = alpha / N
    A = []; lo = []; hi = []
    def add(rr, cc, vv, l, h):
        A.append(sp.csr_matrix((vv, (rr, cc)), shape=(int(max(rr) + 1) if len(rr) else 0, nv))); lo.append(l); hi.append(h)
    # C4
    rr = np.repeat(np.arange(R), N); cc = np.arange(nx)
    add(rr, cc, np.ones(nx), np.ones(R), np.ones(R))
    # x <= c
    rf = np.array([r[0] for r in rows]); rs = np.array([r[1] for r in rows]); rw = np.array([r[2] for r in rows])
    k = np.arange(nx); rowof = k // N; j = k % N
    add(np.concatenate([k, k]), np.concatenate([k, c0 + rf[rowof] * N + j]), np.concatenate([np.ones(nx), -np.ones(nx)]), np.full(nx, -np.inf), np.zeros(nx))
    # c <= n
    q = np.arange(F * N)
    add(np.concatenate([q, q]), np.concatenate([c0 + q, n0 + q % N]), np.concatenate([np.ones(F * N), -np.ones(F * N)]), np.full(F * N, -np.inf), np.zeros(F * N))
    # memory
    add(np.concatenate([q % N, np.arange(N)]), np.concatenate([c0 + q, n0 + np.arange(N)]), np.concatenate([fm[q // N], -nm]), np.full(N, -np.inf), np.zeros(N))
    # CPU
    ld = rs[rowof] >= 0
    wv = np.where(ld, W[rf[rowof], np.maximum(rs[rowof], 0)] * cpr[rf[rowof], j], 0.0)
    sel = wv != 0
    add(np.concatenate([j[sel], np.arange(N)]), np.concatenate([k[sel], n0 + np.arange(N)]), np.concatenate([wv[sel], -cores]), np.full(N, -np.inf), np.zeros(N))
    if c2:
        # colsum - c >= -eps
        add(np.concatenate([rf[rowof] * N + j, q]), np.concatenate([k, c0 + q]), np.concatenate([rw[rowof], -np.ones(F * N)]), np.full(F * N, -1e-6), np.full(F * N, np.inf))
    for e in extra:
        e(add, locals())
    Am = sp.vstack(A).tocsr(); lo = np.concatenate(lo); hi = np.concatenate(hi)
    integ = np.zeros(nv); integ[c0:] = 1
    ub = np.ones(nv)
    return dict(A=Am, lo=lo, hi=hi, c=cost, integ=integ, ub=ub, rows=rows, N=N, F=F, R=R, c0=c0, n0=n0, alpha=alpha,
                W=W, D=D, cpr=cpr, cores=cores, fm=fm, nm=nm, mwd=mwd)

def solve(m, integral, tl=None, opts=None):
    o = {"disp": False}
    if tl: o["time_limit"] = tl
    if opts: o.update(opts)
    t = time.time()
    r = milp(m["c"], constraints=LinearConstraint(m["A"], m["lo"], m["hi"]), bounds=Bounds(0, m["ub"]),
             integrality=m["integ"] if integral else None, options=o)
    return r, time.time() - t

if __name__ == "__main__":
    N, F = int(sys.argv[1]), int(sys.argv[2]); tl = float(sys.argv[3]) if len(sys.argv) > 3 else 300
    m = build(N, F)
    print("R", m["R"], "vars", m["A"].shape, flush=True)
    r, t = solve(m, False)
    n = r.x[m["n0"]:]; print("LP", r.fun, "t", round(t,1), "sum n", n.sum(), "frac n", int(((n > 1e-6) & (n < 1 - 1e-6)).sum()), "delay part", r.fun - m["alpha"] / N * n.sum(), flush=True)
    r2, t2 = solve(m, True, tl, {"disp": False})
    print("MIP", r2.fun, getattr(r2, "mip_dual_bound", None), r2.status, r2.message, "t", round(t2,1), flush=True)
    if r2.x is not None:
        n2 = r2.x[m["n0"]:]; print("  sum n", n2.sum(), "delay", r2.fun - m["alpha"] / N * n2.sum())
