"""ORACLE (test infrastructure only): HiGHS on the restated CSR + the reference's two-step flow.

  solve(model, relax, lb, ub)  one LP relaxation or MIP (HiGHS via scipy.optimize.milp) — stands in
                               for `pywraplp.Solver.Solve()` (`core/solvers/solver.py:35-40`)
  run_flow(payload)            `NeptuneBase.solve/results/score` (`core/solvers/neptune/neptune.py:18-39`):
                               step 1 -> max_score -> step-2 delete -> (if not OPTIMAL) step-2 create,
                               then the wire format of `neptune/utils/output.py:23-39`
  lp_batch_cpu(...)            the CPU baseline leg of bench.py: node LPs of one instance solved by
                               HiGHS, one LP per worker process
"""
import json
import os
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp

from .formulation import build_model
from .inputs import check_input, data_to_solver_input

OPTIMAL, INFEASIBLE = 0, 2
VARIANT = {"NeptuneMinDelayAndUtilization": "MinDelayAndUtilization", "NeptuneMinDelay": "MinDelay",
           "NeptuneMinUtilization": "MinUtilization"}


def solve(m, relax=True, lb=None, ub=None, time_limit=None):
    """Returns (status, objective, x); status 0 = optimal, 2 = infeasible (milp's codes)."""
    integ = np.zeros_like(m["integrality"]) if relax else m["integrality"]
    opts = {"mip_rel_gap": 0.0}
    if time_limit:
        opts["time_limit"] = time_limit
    cons = [LinearConstraint(m["A"], m["lo"], m["hi"])] if m["A"].shape[0] else []
    res = milp(m["c"], constraints=cons, integrality=integ,
               bounds=Bounds(m["lb"] if lb is None else lb, m["ub"] if ub is None else ub), options=opts)
    if res.x is None:
        return int(res.status), None, None
    return int(res.status), float(m["c"] @ res.x), np.asarray(res.x)


def convert_x(xm, nodes, functions):
    """output.py:23-31 — routing[src][fn][dst] = round(x, 3) where x > 0.001."""
    out = {}
    for i, src in enumerate(nodes):
        for f, fn in enumerate(functions):
            for j, dst in enumerate(nodes):
                if xm[i][f][j] > 0.001:
                    out.setdefault(src, {}).setdefault(fn, {})[dst] = float(np.round(xm[i][f][j], 3))
    return json.loads(json.dumps(out))


def convert_c(cm, functions, nodes):
    """output.py:33-39 — alloc[fn][dst] = True where c > 0.001."""
    out = {}
    for f, fn in enumerate(functions):
        for j, dst in enumerate(nodes):
            if cm[f][j] > 0.001:
                out.setdefault(fn, {})[dst] = True
    return out


def _split(m, z, N, F):
    L = m["layout"]
    if z is None:
        z = np.zeros(L.nvars)
    xm = z[:L.nx].reshape(F, N, N).transpose(1, 0, 2)  # -> [i, f, j]
    cm = z[L.c0:L.c0 + F * N].reshape(F, N)
    return xm, cm


def run_flow(payload, time_limit=None):
    """The reference request path (main.py:35-64 minus Flask/timing) on HiGHS."""
    check_input(payload)
    stype = payload.get("solver", {"type": "NeptuneMinDelayAndUtilization"})
    args = dict(stype.get("args", {}))
    variant = VARIANT[stype["type"]]
    data = data_to_solver_input(payload, workload_coeff=payload.get("workload_coeff", 1),
                                with_db=payload.get("with_db", True))
    F, N = data.workload_matrix.shape
    alpha = args.get("alpha", 0.5)
    soften = args.get("soften_step1_sol", 1.3)
    m1 = build_model(data, variant, step=1, alpha=alpha)
    st1, obj1, z1 = solve(m1, relax=False, time_limit=time_limit)
    score1 = obj1 if obj1 is not None else 0.0
    x1, c1 = _split(m1, z1, N, F)
    solved = False
    score2 = 0.0
    x2 = c2 = None
    for mode in ("delete", "create"):
        m2 = build_model(data, variant, step=2, mode=mode, alpha=alpha, soften_step1_sol=soften,
                         max_score=score1, prev_x=x1)
        st2, obj2, z2 = solve(m2, relax=False, time_limit=time_limit)
        score2 = obj2 if obj2 is not None else 0.0
        if st2 == OPTIMAL:
            solved = True
            x2, c2 = _split(m2, z2, N, F)
            break
    xs, cs = (x2, c2) if solved else (x1, c1)
    return {"cpu_routing_rules": convert_x(xs, data.nodes, data.functions),
            "cpu_allocations": convert_c(cs, data.functions, data.nodes),
            "score": {"step1": score1, "step2": score2}}


_POOL_MODEL = None   # the model the forked pool workers inherit (lp_batch_cpu)


def _one_lp(args):
    idx, lo, hi = args
    m = _POOL_MODEL
    lb, ub = m["lb"].copy(), m["ub"].copy()
    lb[idx], ub[idx] = lo, hi
    t = time.perf_counter()
    st, obj, _ = solve(m, relax=True, lb=lb, ub=ub)
    return st, obj, time.perf_counter() - t


def lp_batch_cpu(m, bounds, workers=None):
    """Solve len(bounds) node LPs (lb, ub pairs) of one model, one per worker process.
    Returns (statuses, objectives, wall seconds, workers used).  The workers are forked with the model (not
    pickled per task: a 256x128 model is ~0.4 GB); each task carries its bounds' difference from the model's."""
    import multiprocessing as mp
    global _POOL_MODEL
    workers = workers or os.cpu_count() or 1
    tasks = []
    for lb, ub in bounds:
        idx = np.flatnonzero((lb != m["lb"]) | (ub != m["ub"]))
        tasks.append((idx, lb[idx], ub[idx]))
    _POOL_MODEL = m
    try:
        t0 = time.perf_counter()
        with ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context("fork")) as ex:
            res = list(ex.map(_one_lp, tasks))
        wall = time.perf_counter() - t0
    finally:
        _POOL_MODEL = None
    return [r[0] for r in res], [r[1] for r in res], wall, workers
