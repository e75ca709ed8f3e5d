"""Helpers of the at-scale GPU parity tests (tests/test_gpu_scale.py): the committed HiGHS objectives
of tests/golden/scale.json (tools/gen_scale_golden.py) and an independent host check of an engine
solution against the reference rows (constraints_step1.py / constraints_step2.py)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = os.path.join(HERE, "golden", "scale.json")
VARIANT_CODE = {"MinDelay": 0, "MinUtilization": 1, "MinDelayAndUtilization": 2}


def scale_cases():
    with open(SCALE) as fh:
        return json.load(fh)


def case_payload(c):
    if c["kind"] == "synthetic":
        from core.utils.synthetic import synthetic_payload
        return synthetic_payload(c["N"], c["F"], seed=c["seed"])
    with open(os.path.join(HERE, "golden", "inputs", c["input"] + ".json")) as fh:
        return json.load(fh)


def case_model_args(c):
    """(data, variant, step, kwargs of core.engine.lp.LPModel) of a scale.json case."""
    from core.utils import data_to_solver_input
    p = case_payload(c)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    kw = {"alpha": alpha}
    if c["step"] != 1:
        kw.update(max_score=c["max_score"], soften_step1_sol=1.3)
    return data, c["variant"], c["step"], kw


def node_bounds(c, n_int):
    """[B, n_int] bound arrays of the case's node fixings (-inf / +inf where free)."""
    B = len(c["nodes"])
    lb = np.full((B, n_int), -np.inf)
    ub = np.full((B, n_int), np.inf)
    for b, nd in enumerate(c["nodes"]):
        lb[b, nd["fix_idx"]] = nd["fix_val"]
        ub[b, nd["fix_idx"]] = nd["fix_val"]
    return lb, ub


def gap(a, b):
    return abs(a - b) / max(1.0, abs(b))


def check_step1_solution(data, variant, alpha, xb, row_f, row_src, z, lb=None, ub=None, tol=1e-6, simplex_tol=2e-5):
    """Independent fp64 host check of a step-1 engine solution (aggregated routing rows xbar[R, N],
    row map, integer vector z = c[F*N] (+ n[N])) against the reference rows:
      C4 (constraints_step1.py:27-34)  sum_j x[i,f,j] = 1 per routing row (fp32 state: simplex_tol)
      C1/C2 (:5-15)   flow[f,j] - M c[f,j] <= 0,  flow[f,j] - c[f,j] >= -eps
      C3 (:18-23)     sum_f mem_f c[f,j] <= Mem_j
      C5 (:57-65)     sum_{f,i} W[f,i] cpr[f,j] x[i,f,j] <= cores_j
      C6/C7 (:69-78)  sum_f c - M n <= 0, sum_f c - n >= -eps
    Returns (max normalised violation, objective recomputed from x and z, objectives.py:4-53)."""
    W = np.asarray(data.workload_matrix, np.float64)
    D = np.asarray(data.node_delay_matrix, np.float64)
    cpr = np.asarray(data.core_per_req_matrix, np.float64)
    F, N = W.shape
    M, eps = 1e6, 1e-6
    x = np.asarray(xb, np.float64)
    zero_src = (W == 0).sum(axis=1).astype(np.float64)
    wrow = np.where(row_src >= 0, 1.0, zero_src[row_f])
    viol = {}
    viol["C4"] = float(np.abs(x.sum(axis=1) - 1.0).max()) if len(x) else 0.0
    viol["xneg"] = float(max(0.0, -x.min())) if len(x) else 0.0
    flow = np.zeros((F, N))
    np.add.at(flow, row_f, wrow[:, None] * x)
    c = np.asarray(z[:F * N], np.float64).reshape(F, N)
    has_n = variant != "MinDelay"
    viol["C1"] = float(np.maximum(flow - M * c, 0).max() / M)
    viol["C2"] = float(np.maximum(-(flow - c) - eps, 0).max())
    mem = (np.asarray(data.function_memory_matrix, np.float64)[:, None] * c).sum(axis=0)
    nm = np.asarray(data.node_memory_matrix, np.float64)
    viol["C3"] = float((np.maximum(mem - nm, 0) / np.maximum(1.0, nm)).max())
    wsrc = np.where(row_src >= 0, W[row_f, np.maximum(row_src, 0)], 0.0)
    cpu = np.zeros(N)
    for f in range(F):
        sel = row_f == f
        if sel.any():
            cpu += cpr[f] * (wsrc[sel, None] * x[sel]).sum(axis=0)
    cores = np.asarray(data.node_cores_matrix, np.float64)
    viol["C5"] = float((np.maximum(cpu - cores, 0) / np.maximum(1.0, cores)).max())
    obj = 0.0
    if has_n:
        n = np.asarray(z[F * N:F * N + N], np.float64)
        sc = c.sum(axis=0)
        viol["C6"] = float(np.maximum(sc - M * n, 0).max() / M)
        viol["C7"] = float(np.maximum(-(sc - n) - eps, 0).max())
    for nm_, lim in (("lb", lb), ("ub", ub)):
        if lim is not None:
            zz = np.asarray(z, np.float64)
            fin = np.isfinite(lim)
            d = (lim[fin] - zz[fin]) if nm_ == "lb" else (zz[fin] - lim[fin])
            viol[nm_] = float(max(0.0, d.max())) if d.size else 0.0
    # objective (objectives.py:4-53)
    dsrc = np.where(row_src[:, None] >= 0, D[np.maximum(row_src, 0)], 0.0)
    xdelay = (wsrc[:, None] * dsrc * x).sum()
    if variant == "MinDelay":
        obj = xdelay
    elif variant == "MinUtilization":
        obj = float(np.sum(z[F * N:F * N + N]))
    else:
        obj = alpha / N * float(np.sum(z[F * N:F * N + N]))
        if W.sum():
            md = np.asarray(data.max_delay_matrix, np.float64)
            mwd = 0.0                     # objectives.py:36-43, vectorised over the distinct max delays
            for mdv in np.unique(md):
                best = np.where(D <= mdv, D, -np.inf).max(axis=1)
                mwd += float((W[md == mdv] * best[None, :]).sum())
            obj += (1 - alpha) * xdelay / mwd
    worst = max(v for k, v in viol.items() if k != "C4")
    return viol, worst, obj


def check_step2_solution(data, variant, alpha, mode, max_score, xb, row_f, row_src, z, lb=None, ub=None,
                         soften=1.3, prev_delay=0.0, tol=1e-6, simplex_tol=2e-5):
    """Independent fp64 host check of a step-2 engine solution: the step-1 rows C1-C7 (check_step1_solution,
    on c and n) plus the step-2 rows of constraints_step2.py and the disruption objective
    (objectives.py:55-63).  z = c, moved_from, moved_to [F*N each], allocated, deallocated (+ n[N]):
      D1 (:5-9)    mf >= 0, mf - c >= -old          D2 (:12-16)  mt >= 0, mt + c >= old
      D3 (:19-33)  a <= 0, sumOld - sum c >= a, d <= 0, sum c - sumOld >= d
      D4 (:36-55)  delete: d + a + sumOld - sum c >= 0 ; create: d + a - sumOld + sum c >= 0
      D5/D6/D7 (:57-88) the variant's score row (normalised by its right-hand side)
    Returns (violations, worst, disruption objective recomputed from z)."""
    W = np.asarray(data.workload_matrix, np.float64)
    F, N = W.shape
    FN = F * N
    z = np.asarray(z, np.float64)
    has_n = variant != "MinDelay"
    c, mf, mt = z[:FN], z[FN:2 * FN], z[2 * FN:3 * FN]
    a, d = float(z[3 * FN]), float(z[3 * FN + 1])
    n = z[3 * FN + 2:3 * FN + 2 + N] if has_n else np.zeros(0)
    z1 = np.concatenate([c, n])
    box1 = [None, None]
    for k, lim in enumerate((lb, ub)):
        if lim is not None:
            lim = np.asarray(lim, np.float64)
            box1[k] = np.concatenate([lim[:FN], lim[3 * FN + 2:3 * FN + 2 + N] if has_n else np.zeros(0)])
    viol, _, _ = check_step1_solution(data, variant if has_n else "MinDelay", alpha, xb, row_f, row_src, z1,
                                      box1[0], box1[1], tol, simplex_tol)
    old = np.asarray(data.old_allocations_matrix, np.float64).ravel()
    so, sc = float(old.sum()), float(c.sum())
    viol["D1"] = float(max(0.0, (-mf).max(), (-(mf - c) - old).max()))
    viol["D2"] = float(max(0.0, (-mt).max(), (old - (mt + c)).max()))
    viol["D3"] = float(max(0.0, a, a - (so - sc), d, d - (sc - so)) / max(1.0, so))
    d4 = (d + a + so - sc) if mode == "delete" else (d + a - so + sc)
    viol["D4"] = float(max(0.0, -d4) / max(1.0, so))
    x = np.asarray(xb, np.float64)
    D = np.asarray(data.node_delay_matrix, np.float64)
    wsrc = np.where(row_src >= 0, W[row_f, np.maximum(row_src, 0)], 0.0)
    dsrc = np.where(row_src[:, None] >= 0, D[np.maximum(row_src, 0)], 0.0)
    if variant == "MinUtilization":
        lhs, rhs = float(n.sum()), max_score * soften
    elif variant == "MinDelay":
        lhs, rhs = float((wsrc[:, None] * dsrc * x).sum()), soften * prev_delay
    else:
        md = np.maximum(np.asarray(data.max_delay_matrix, np.float64)[None, :], D.max(axis=0)[:, None])  # [i, f]
        mdr = np.where(row_src >= 0, md[np.maximum(row_src, 0), row_f], 1.0)
        lhs = alpha / N * float(n.sum()) + float((((1 - alpha) * wsrc / mdr)[:, None] * dsrc * x).sum())
        rhs = max_score * soften
    viol["score"] = float(max(0.0, lhs - rhs) / max(1.0, abs(rhs)))
    if lb is not None:
        viol["lb"] = float(max(0.0, np.nanmax(np.where(np.isfinite(lb), np.asarray(lb) - z, 0.0))))
    if ub is not None:
        viol["ub"] = float(max(0.0, np.nanmax(np.where(np.isfinite(ub), z - np.asarray(ub), 0.0))))
    w = float(FN)
    obj = w * float(mf.sum() + mt.sum()) + (w - 1) * a + (w + 1) * d
    worst = max(v for k, v in viol.items() if k != "C4")
    return viol, worst, obj
