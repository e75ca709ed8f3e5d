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
