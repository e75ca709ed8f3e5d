"""Primal heuristics of the branch-and-bound (core/engine/bnb.py) that need the instance's data.

`capacity_greedy` — a leaf (every c and n fixed) that is feasible by construction for the reference's rows:
open nodes in the order an LP ranks them (the node values n of the facility relaxation), then
route every loaded source of every function, heaviest first, to the open node of least delay that still has
CPU room for it (constraints_step1.py:57-65) and memory for the function (:18-23), opening that placement;
a function without loaded sources gets the open node with memory room the LP prefers.  Every open
placement then carries >= 1 unit of flow (C2, :5-15) and every source is routed (C4, :27-34), so the leaf LP
has a feasible point — the greedy routing itself; more nodes are opened until the routing succeeds.  The
node box's fixings are kept (closed nodes / placements excluded, fixed-open ones opened first).
"""
import numpy as np


def capacity_greedy(W, D, cpr, cores, fmem, nmem, n_rank, flow=None, start=None, step=None, tries=4,
                    node_cost=0.0, delay_coef=0.0, c_fix=None, n_fix=None, new_pen=0.5):
    """Leaves [(c [F, N] 0/1, n [N] 0/1, estimate, route)], best estimate first (at most `tries`, one per node
    count); route = (f, i, j) arrays: the loaded source i of f sends all of its workload to j.

    W [F, N] workload, D [N, N] delay, cpr [F, N], cores [N], fmem [F], nmem [N]; n_rank [N]: the order in
    which nodes are opened (descending); flow [F, N] (optional): the LP's flows, tie-break among equal delays.
    start: nodes opened first (default: enough cores for the total CPU demand at each function's cheapest
    cpr); step: nodes added per retry.  estimate = node_cost * open nodes + delay_coef * sum W D of the greedy
    routing (the objective of a feasible point of the leaf, so an upper bound on its LP value).
    c_fix [F, N] / n_fix [N]: -1 free, 0 / 1 fixed (the node's box).  new_pen: a new placement is charged
    new_pen x the median delay between open nodes in the routing choice."""
    W = np.asarray(W, np.float64)
    F, N = W.shape
    D = np.asarray(D, np.float64)
    cpr = np.asarray(cpr, np.float64)
    cores = np.asarray(cores, np.float64)
    fmem = np.asarray(fmem, np.float64)
    nmem = np.asarray(nmem, np.float64)
    rank = np.asarray(n_rank, np.float64).copy()
    cfx = np.full((F, N), -1.0) if c_fix is None else np.asarray(c_fix, np.float64).reshape(F, N)
    nfx = np.full(N, -1.0) if n_fix is None else np.asarray(n_fix, np.float64).reshape(N)
    forced = (nfx == 1.0) | (cfx == 1.0).any(axis=0)
    rank[forced] = np.inf
    allowed_j = nfx != 0.0
    order = [j for j in np.lexsort((-cores, -rank)) if allowed_j[j]]
    nf = int(forced.sum())
    fs, src = np.nonzero(W > 0)
    load = W[fs, src]
    rows = np.argsort(-load, kind="stable")
    demand = float((W * np.where(cfx == 0.0, np.inf, cpr).min(axis=1, keepdims=True)).sum())
    if start is None:
        cum = np.cumsum(cores[order])
        start = int(np.searchsorted(cum, demand)) + 1
    step = step or max(1, N // 32)
    k = max(1, nf, min(start, len(order)))
    fl = None if flow is None else np.asarray(flow, np.float64).reshape(F, N)
    out = []
    while k <= len(order) and len(out) < tries:
        openj = np.asarray(order[:k])
        is_open = np.zeros(N, bool)
        is_open[openj] = True
        cap = cores.copy()
        mem = nmem.copy()
        C = np.zeros((F, N))
        ok = True
        for f, j in zip(*np.nonzero(cfx == 1.0)):                  # fixed-open placements first
            if not is_open[j] or fmem[f] > mem[j] + 1e-12:
                ok = False
                break
            C[f, j] = 1.0
            mem[j] -= fmem[f]
        delay = 0.0
        rf, ri, rj = [], [], []
        pen = new_pen * float(np.median(D[np.ix_(openj, openj)])) if k > 1 else 0.0
        for r in rows if ok else ():
            f, i = int(fs[r]), int(src[r])
            need = load[r] * cpr[f]                               # CPU at each destination
            fit = is_open & (cfx[f] != 0.0) & (need <= cap + 1e-12) & ((C[f] > 0) | (fmem[f] <= mem + 1e-12))
            if not fit.any():
                ok = False
                break
            # least delay, a new placement charged `pen` (memory is the scarce resource: a function spread over
            # every open node crowds the others out)
            key = np.where(fit, D[i] + pen * (C[f] == 0), np.inf)
            best = np.flatnonzero(key == key.min())
            j = int(best[np.argmax(fl[f, best])] if fl is not None and len(best) > 1 else best[0])
            cap[j] -= need[j]
            delay += load[r] * D[i, j]
            rf.append(f)
            ri.append(i)
            rj.append(j)
            if C[f, j] == 0:
                C[f, j] = 1.0
                mem[j] -= fmem[f]
        if ok:
            for f in np.flatnonzero(C.sum(axis=1) < 1):             # functions with no loaded source
                cand = np.flatnonzero(is_open & (cfx[f] != 0.0) & (fmem[f] <= mem + 1e-12))
                if cand.size == 0:
                    ok = False
                    break
                j = int(cand[np.argmax(rank[cand] if fl is None else fl[f, cand])])
                C[f, j] = 1.0
                mem[j] -= fmem[f]
        if ok:
            n = (C.sum(axis=0) > 0).astype(np.float64)
            n[nfx == 1.0] = 1.0
            out.append((C, n, node_cost * float(n.sum()) + delay_coef * delay,
                        (np.asarray(rf, np.int64), np.asarray(ri, np.int64), np.asarray(rj, np.int64))))
        k += step
    out.sort(key=lambda t: t[2])
    return out
