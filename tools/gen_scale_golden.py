#!/usr/bin/env python3
"""Golden LP objectives at the BASELINE.json sizes (build container only; writes
tests/golden/scale.json).

For every case: the root LP relaxation of the reference model (oracle/formulation.py, the
reference's builders restated entry by entry and pinned by tests/test_oracle_formulation.py) and
seeded B&B-node relaxations (a few binaries fixed), solved by HiGHS (oracle/solve.py).  Cases:
  * the synthetic generator of SURVEY.md §8(d) (core/utils/synthetic.py) at 64x32 (BASELINE config 2),
    128x64 and 256x128 (config 3), step-1 MinDelayAndUtilization (alpha 0.5), plus step 1 of the other
    two variants and step-2 create/delete models at 64x32;
  * the reference's Alibaba 100x25 trace case (tests/golden/inputs/alibaba_*.json, W == 0: the engine's
    R = F aggregation path), step 1 of all three variants and the step-2 create model at the published
    step-1 scores (testing/alibaba/alibaba_test/output_*_case0.json).
Fixings are indices into the engine's integer vector z_int (include/neptune_lp.h), which is the
reference variable vector minus x: reference index = N*N*F + k.

  python3 tools/gen_scale_golden.py [--workers 3] [--only 64x32,alibaba]
"""
import argparse
import json
import os
import sys
import time
import zlib
from concurrent.futures import ProcessPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden", "scale.json")
ALIBABA_PUBLISHED_STEP1 = {"NeptuneMinDelayAndUtilization": 0.005, "NeptuneMinDelay": 0.0,
                           "NeptuneMinUtilization": 1.0}


def cases():
    out = []
    for (n, f) in ((64, 32), (128, 64), (256, 128)):
        out.append(dict(name=f"syn{n}x{f}_MDU_s1", kind="synthetic", N=n, F=f, seed=0,
                        variant="MinDelayAndUtilization", step=1, children=8))
    for v in ("MinDelay", "MinUtilization"):
        out.append(dict(name=f"syn64x32_{v}_s1", kind="synthetic", N=64, F=32, seed=0, variant=v, step=1, children=4))
    for mode, step in (("create", 3), ("delete", 2)):
        out.append(dict(name=f"syn64x32_MDU_s2{mode}", kind="synthetic", N=64, F=32, seed=0,
                        variant="MinDelayAndUtilization", step=step, mode=mode, max_score=0.05, children=4))
        # round 5: more step-2 models (the reduced disruption block) — MinUtilization at 64x32 and
        # MinDelayAndUtilization at 128x64, seed 1
        out.append(dict(name=f"syn64x32_MU_s2{mode}", kind="synthetic", N=64, F=32, seed=0,
                        variant="MinUtilization", step=step, mode=mode, max_score=8.0, children=4))
        out.append(dict(name=f"syn128x64_MDU_s2{mode}", kind="synthetic", N=128, F=64, seed=1,
                        variant="MinDelayAndUtilization", step=step, mode=mode, max_score=2.0, children=4))
    for t, v in (("NeptuneMinDelayAndUtilization", "MinDelayAndUtilization"), ("NeptuneMinDelay", "MinDelay"),
                 ("NeptuneMinUtilization", "MinUtilization")):
        out.append(dict(name=f"alibaba_{v}_s1", kind="alibaba", input=f"alibaba_{t}", variant=v, step=1, children=6))
        if v != "MinDelay":
            out.append(dict(name=f"alibaba_{v}_s2create", kind="alibaba", input=f"alibaba_{t}", variant=v, step=3,
                            mode="create", max_score=ALIBABA_PUBLISHED_STEP1[t], children=4))
    return out


def payload_of(c):
    if c["kind"] == "synthetic":
        from core.utils.synthetic import synthetic_payload
        return synthetic_payload(c["N"], c["F"], seed=c["seed"])
    with open(os.path.join(REPO, "tests", "golden", "inputs", c["input"] + ".json")) as fh:
        return json.load(fh)


def model_of(c):
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input
    p = payload_of(c)
    d = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    if c["step"] == 1:
        m = build_model(d, c["variant"], step=1, alpha=alpha)
    else:
        m = build_model(d, c["variant"], step=2, mode=c["mode"], alpha=alpha, max_score=c["max_score"],
                        soften_step1_sol=1.3)
    return m, d


def fixings(c, n_int, F, N):
    """Seeded node fixings: children 0..k/2-1 fix 2 c[f,j]; the rest fix 6 (c and, with n, n[j])."""
    rng = np.random.default_rng(zlib.crc32(c["name"].encode()))
    has_n = c["variant"] != "MinDelay"
    n0 = (F * N if c["step"] == 1 else 3 * F * N + 2) if has_n else None
    out = []
    for b in range(c["children"]):
        k = 2 if b < c["children"] // 2 else 6
        idx = rng.choice(F * N, size=k, replace=False).tolist()
        if has_n and b >= c["children"] // 2:
            idx[-1] = n0 + int(rng.integers(0, N))
        val = rng.integers(0, 2, size=k).astype(float).tolist()
        out.append((idx, val))
    return out


def solve_one(args):
    c, b = args
    from oracle.solve import solve
    t0 = time.time()
    m, d = model_of(c)
    F, N = d.workload_matrix.shape
    nx = N * N * F
    n_int = m["c"].shape[0] - nx
    if b < 0:
        st, obj, _ = solve(m, relax=True)
        return c["name"], b, None, None, (obj if st == 0 else None), st, time.time() - t0, n_int
    idx, val = fixings(c, n_int, F, N)[b]
    lb, ub = m["lb"].copy(), m["ub"].copy()
    for i, v in zip(idx, val):
        lb[nx + i] = ub[nx + i] = v
    st, obj, _ = solve(m, relax=True, lb=lb, ub=ub)
    return c["name"], b, idx, val, (obj if st == 0 else None), st, time.time() - t0, n_int


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    cs = cases()
    if a.only:
        keys = a.only.split(",")
        cs = [c for c in cs if any(k in c["name"] for k in keys)]
    old = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            old = json.load(fh)
    tasks = [(c, b) for c in cs for b in range(-1, c["children"])]
    # big ones first
    tasks.sort(key=lambda t: -(t[0].get("N", 100) ** 2 * t[0].get("F", 25)))
    res = {}
    with ProcessPoolExecutor(max_workers=a.workers) as ex:
        for name, b, idx, val, obj, st, sec, n_int in ex.map(solve_one, tasks):
            print(f"{name} node {b}: status {st} obj {obj} ({sec:.1f}s)", flush=True)
            res.setdefault(name, {})[b] = (idx, val, obj, st, sec, n_int)
    for c in cs:
        r = res[c["name"]]
        entry = {k: v for k, v in c.items() if k != "children"}
        entry["n_int"] = r[-1][5]
        entry["root"] = {"lp_objective": r[-1][2], "status": r[-1][3], "highs_seconds": round(r[-1][4], 2)}
        entry["nodes"] = [{"fix_idx": r[b][0], "fix_val": r[b][1], "lp_objective": r[b][2], "status": r[b][3],
                           "highs_seconds": round(r[b][4], 2)} for b in range(c["children"])]
        old[c["name"]] = entry
    with open(OUT, "w") as fh:
        json.dump(old, fh, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
