#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run in the BUILD container only).

How: the reference's own model builders (`/root/reference/core/**`) are imported unmodified
with two probe-only stand-ins ahead of them on sys.path (tools/refshim: a recording
`pywraplp` whose Solve() is HiGHS via scipy, and `hurry.filesize`).  Every model the
reference builds is recorded as CSR (A, row bounds, objective, variable bounds,
integrality) and solved by HiGHS — as MIP (the reference flow) and as LP relaxation.

Outputs (data only — no reference source is copied):
  tests/golden/inputs/<case>.json        REST payloads (comment-stripped payload.json, test.py's
                                         input, seeded synthetic payloads, Alibaba trace input)
  tests/golden/models/<case>__<k>.npz    recorded reference model k of that case (tiny cases)
  tests/golden/golden.json               per case: reference response (score/allocations/routing),
                                         per-model LP & MIP objectives, node-LP objectives under
                                         seeded bound fixings, uniqueness flags, provenance.

The reference cannot travel to the GPU box; these fixtures do.
Usage:  python tools/gen_golden.py [--alibaba] [--quick]
"""
import argparse
import ast
import contextlib
import importlib.util
import io
import json
import os
import re
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")

sys.dont_write_bytecode = True  # the reference tree is read-only
sys.path[:0] = [os.path.join(HERE, "refshim"), REF]

from ortools.linear_solver import pywraplp  # noqa: E402  (the stand-in)
from core import data_to_solver_input, check_input  # noqa: E402  (the reference)
import core.solvers as RS  # noqa: E402
from scipy.optimize import Bounds, LinearConstraint, milp  # noqa: E402


def _load_product_module(rel, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


synthetic = _load_product_module("neptune-mip_amd/core/utils/synthetic.py", "nep_synthetic")


def strip_comments(text):
    return "\n".join(re.sub(r"\s*//.*$", "", line) for line in text.splitlines())


def solve_model(m, relax, extra_lb=None, extra_ub=None, time_limit=None):
    """HiGHS on a recorded model; returns (status, objective-in-model-sense, x)."""
    c = -m["c"] if m["maximize"] else m["c"]
    lb = m["lb"] if extra_lb is None else extra_lb
    ub = m["ub"] if extra_ub is None else extra_ub
    integ = np.zeros_like(m["integrality"]) if relax else m["integrality"]
    opts = {"mip_rel_gap": 0.0}
    if time_limit:
        opts["time_limit"] = time_limit
    cons = [LinearConstraint(m["A"], m["lo"], m["hi"])] if m["A"].shape[0] else []
    res = milp(c, constraints=cons, integrality=integ, bounds=Bounds(lb, ub), options=opts)
    if res.x is None:
        return int(res.status), None, None
    obj = float(m["offset"] + m["c"] @ res.x)
    return int(res.status), obj, res.x


def run_reference(payload, quiet=True):
    """The reference flow (main.py:35-51 minus Flask) with the recorder installed."""
    pywraplp.Solver.RECORD = []
    pywraplp.Solver.RELAX = False
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        check_input(payload)
        solver_cfg = payload.get("solver", {"type": "NeptuneMinDelayAndUtilization"})
        cls = getattr(RS, solver_cfg["type"])
        s = cls(**solver_cfg.get("args", {}))
        data = data_to_solver_input(payload, with_db=payload.get("with_db", True),
                                    workload_coeff=payload.get("workload_coeff", 1))
        s.load_data(data)
        s.solve()
        x, c = s.results()
        score = s.score()
    elapsed = time.time() - t0
    models = pywraplp.Solver.RECORD
    pywraplp.Solver.RECORD = None
    return {"cpu_routing_rules": x, "cpu_allocations": c, "score": score}, models, data, elapsed


def model_summary(m):
    return {"n_vars": int(m["A"].shape[1]), "n_rows": int(m["A"].shape[0]), "nnz": int(m["A"].nnz),
            "status": int(m["status"]), "mip_objective": m["objective"]}


def tie_check(m):
    """Re-solve the MIP with a no-good cut on the binary vector of its optimum."""
    if m["x"] is None or m["status"] != 0:
        return None
    integ = m["integrality"].astype(bool)
    binary = integ & (m["lb"] == 0) & (m["ub"] == 1)
    idx = np.nonzero(binary)[0]
    xs = np.rint(m["x"][idx])
    row = np.zeros(m["A"].shape[1])
    row[idx] = np.where(xs > 0.5, -1.0, 1.0)
    rhs = 1.0 - float((xs > 0.5).sum())
    import scipy.sparse as sp
    A2 = sp.vstack([m["A"], sp.csr_matrix(row)]).tocsr()
    m2 = dict(m)
    m2["A"] = A2
    m2["lo"] = np.append(m["lo"], rhs)
    m2["hi"] = np.append(m["hi"], np.inf)
    st, obj, _ = solve_model(m2, relax=False, time_limit=120)
    if obj is None:
        return True
    return bool(abs(obj - m["objective"]) <= 1e-7 * max(1.0, abs(m["objective"])))


def node_fixings(m, rng, k):
    """Seeded B&B-node style bound fixings on binary vars; HiGHS LP objective for each."""
    integ = m["integrality"].astype(bool)
    binary = np.nonzero(integ & (m["lb"] == 0) & (m["ub"] == 1))[0]
    out = []
    for _ in range(k):
        lb, ub = m["lb"].copy(), m["ub"].copy()
        nfix = int(rng.integers(1, max(2, len(binary) // 3) + 1))
        pick = rng.choice(binary, size=min(nfix, len(binary)), replace=False)
        vals = rng.integers(0, 2, size=len(pick))
        lb[pick] = vals
        ub[pick] = vals
        st, obj, _ = solve_model(m, relax=True, extra_lb=lb, extra_ub=ub)
        out.append({"fix_idx": pick.tolist(), "fix_val": vals.tolist(), "status": st, "lp_objective": obj})
    return out


def save_model(path, m, lp_obj, lp_x):
    A = m["A"].tocsr()
    np.savez_compressed(
        path, A_data=A.data, A_indices=A.indices.astype(np.int32), A_indptr=A.indptr.astype(np.int64),
        A_shape=np.array(A.shape, np.int64), lo=m["lo"], hi=m["hi"], c=m["c"], lb=m["lb"], ub=m["ub"],
        integrality=m["integrality"], names=np.array(m["names"], dtype=np.str_),
        maximize=np.array(m["maximize"]), offset=np.array(m["offset"]),
        mip_status=np.array(m["status"]), mip_objective=np.array(np.nan if m["objective"] is None else m["objective"]),
        mip_x=(m["x"] if m["x"] is not None else np.zeros(0)),
        lp_objective=np.array(np.nan if lp_obj is None else lp_obj), lp_x=(lp_x if lp_x is not None else np.zeros(0)))


def do_case(name, payload, golden, save_models=True, fixings=6, check_ties=True, seed=0):
    print(f"[{name}] running reference flow ...", flush=True)
    resp, models, data, elapsed = run_reference(payload)
    entry = {"response": resp, "elapsed_s": round(elapsed, 3), "models": []}
    rng = np.random.default_rng(seed)
    for k, m in enumerate(models):
        st, lp_obj, lp_x = solve_model(m, relax=True)
        s = model_summary(m)
        s["lp_status"] = st
        s["lp_objective"] = lp_obj
        s["mode"] = ["step1", "step2_delete", "step2_create"][k] if k < 3 else f"model{k}"
        if check_ties and m["A"].shape[1] <= 5000:
            s["mip_tied"] = tie_check(m)
        if fixings and m["A"].shape[1] <= 5000:
            s["node_lps"] = node_fixings(m, rng, fixings)
        if save_models:
            save_model(os.path.join(OUT, "models", f"{name}__{k}.npz"), m, lp_obj, lp_x)
        entry["models"].append(s)
        print(f"   model {k}: {s['n_vars']} vars {s['n_rows']} rows mip={s['mip_objective']} lp={lp_obj} "
              f"tied={s.get('mip_tied')}", flush=True)
    golden[name] = entry
    with open(os.path.join(OUT, "inputs", f"{name}.json"), "w") as f:
        json.dump(payload, f)


def testpy_payload():
    """The request literal of `test.py:5-55` (+ :57-58), parsed as data via ast."""
    src = open(os.path.join(REF, "test.py")).read()
    tree = ast.parse(src)
    payload = None
    for node in tree.body:
        if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", None) == "input":
            payload = ast.literal_eval(node.value)
    n_f = len(payload["function_names"])
    payload["cores_matrix"] = [[1, 1, 1]] * n_f
    payload["workload_on_destination_matrix"] = [[1, 1, 1]] * n_f
    return payload


def simulated_payloads():
    """The 10 request literals of `testing/simulated/simulated_test.py:25-380`, evaluated as data
    (they use list comprehensions, so ast.literal_eval is not enough)."""
    src = open(os.path.join(REF, "testing/simulated/simulated_test.py")).read()
    tree = ast.parse(src)
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", None) == "inputs":
            expr = ast.Expression(node.value)
            out = {}
            for st in ["NeptuneMinDelayAndUtilization", "NeptuneMinDelay", "NeptuneMinUtilization"]:
                out[st] = eval(compile(expr, "simulated_inputs", "eval"), {"__builtins__": {"range": range}},
                               {"solver_type": st})
            return out
    raise RuntimeError("inputs literal not found")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alibaba", action="store_true", help="also record the Alibaba 100x25 step-1 LPs")
    ap.add_argument("--simulated", action="store_true", help="also run simulated cases 0-6 through the MIP")
    args = ap.parse_args()
    os.makedirs(os.path.join(OUT, "models"), exist_ok=True)
    os.makedirs(os.path.join(OUT, "inputs"), exist_ok=True)
    gpath = os.path.join(OUT, "golden.json")
    golden = json.load(open(gpath)) if os.path.exists(gpath) else {}

    # 1. payload.json (comment-stripped; with_db=false: the DB path is out of scope)
    payload = json.loads(strip_comments(open(os.path.join(REF, "payload.json")).read()))
    payload["with_db"] = False
    do_case("payload", payload, golden)

    # 2. test.py request -> output-mip.json (SCIP output committed in the reference)
    tp = testpy_payload()
    do_case("testpy", tp, golden)
    scip_out = json.loads(open(os.path.join(REF, "output-mip.json")).read().replace("True", "true"))
    golden["testpy"]["scip_response"] = scip_out

    # 3. seeded synthetic payloads (tiny), each solver variant
    for (N, F, seed, rho) in [(4, 3, 0, 0.5), (6, 4, 1, 0.3), (8, 4, 2, 0.1), (8, 4, 3, 1.0), (10, 5, 4, 0.2)]:
        for st in ["NeptuneMinDelayAndUtilization", "NeptuneMinDelay", "NeptuneMinUtilization"]:
            p = synthetic.synthetic_payload(N, F, seed=seed, rho=rho, solver_type=st)
            do_case(f"syn_{N}x{F}_s{seed}_r{rho}_{st}", p, golden, seed=seed)
        json.dump(golden, open(gpath, "w"), indent=1, default=float)

    # 4. simulated cases 0-4 (tiny; published node counts in the PDF)
    if args.simulated:
        sims = simulated_payloads()
        for st, cases in sims.items():
            for i, p in enumerate(cases):
                if i > 6:
                    continue
                do_case(f"sim{i}_{st}", p, golden, save_models=i <= 4, fixings=0, check_ties=False)
                json.dump(golden, open(gpath, "w"), indent=1, default=float)

    # 5. Alibaba 100x25: published SCIP responses + recorded step-1 LP relaxation objectives
    if args.alibaba:
        adir = os.path.join(REF, "testing/alibaba/alibaba_test")
        for st in ["NeptuneMinDelayAndUtilization", "NeptuneMinDelay", "NeptuneMinUtilization"]:
            d = json.load(open(os.path.join(adir, f"output_{st}_case0.json")))
            inp = d["input"]
            name = f"alibaba_{st}"
            with open(os.path.join(OUT, "inputs", f"{name}.json"), "w") as f:
                json.dump(inp, f)
            step1_cls = {"NeptuneMinDelayAndUtilization": RS.NeptuneStep1CPUMinDelayAndUtilization,
                         "NeptuneMinDelay": RS.NeptuneStep1CPUMinDelay,
                         "NeptuneMinUtilization": RS.NeptuneStep1CPUMinUtilization}[st]
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                data = data_to_solver_input(inp, with_db=False, workload_coeff=inp.get("workload_coeff", 1))
                s1 = step1_cls(**inp["solver"]["args"])
                s1.load_data(data)
                s1.init_objective()
                m = s1.solver.model_arrays()
            t0 = time.time()
            stt, lp_obj, _ = solve_model(m, relax=True)
            print(f"[{name}] step-1 LP {m['A'].shape} nnz={m['A'].nnz} lp={lp_obj} ({time.time()-t0:.1f}s)")
            golden[name] = {
                "published_response": {k: d[k] for k in ["cpu_allocations", "cpu_routing_rules", "score",
                                                          "processing_time"]},
                "step1_model": {"n_vars": int(m["A"].shape[1]), "n_rows": int(m["A"].shape[0]),
                                "nnz": int(m["A"].nnz), "lp_status": stt, "lp_objective": lp_obj},
            }
            json.dump(golden, open(gpath, "w"), indent=1, default=float)

    json.dump(golden, open(gpath, "w"), indent=1, default=float)
    print("wrote", gpath)


if __name__ == "__main__":
    main()
