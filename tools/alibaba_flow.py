#!/usr/bin/env python3
"""The reference's Alibaba 100x25 trace case through the product solvers on the MI355X engine,
against the responses the reference recorded with SCIP
(testing/alibaba/alibaba_test/output_{NeptuneMinDelay,NeptuneMinDelayAndUtilization,
NeptuneMinUtilization}_case0.json; scores 0.0 / 23.0, 0.005 / 65010, 1.0 / 65010; processing_time
436 / 1258 / 1225 s).  Each step's B&B gets `--step-seconds` of wall time; the JSON written to
--out records the scores, B&B statistics (status, bound, nodes, LPs) and wall time per step.

  python3 tools/alibaba_flow.py --step-seconds 120 --out profiles/r02/alibaba_flows.json
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

PUBLISHED = {"NeptuneMinDelay": ({"step1": 0.0, "step2": 23.0}, 436.445),
             "NeptuneMinDelayAndUtilization": ({"step1": 0.005, "step2": 65010.0}, 1258.109),
             "NeptuneMinUtilization": ({"step1": 1.0, "step2": 65010.0}, 1224.564)}


def run(stype, seconds, batch):
    import core.solvers as S
    from core.utils import data_to_solver_input
    with open(os.path.join(REPO, "tests", "golden", "inputs", f"alibaba_{stype}.json")) as fh:
        p = json.load(fh)
    args = dict(p["solver"].get("args", {}))
    args.update(time_limit=seconds, batch=batch, verbose=False, node_limit=10 ** 9)
    t0 = time.time()
    solver = S.SOLVERS[stype](**args)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver.load_data(data)
    solved = solver.solve()
    x, c = solver.results()
    score = solver.score()
    wall = time.time() - t0
    steps = {}
    for k in ("step1", "step2_delete", "step2_create"):
        st = getattr(solver, k)
        r = getattr(st, "result", None)
        if r is not None:
            steps[k] = r.as_dict()
    ref, ref_t = PUBLISHED[stype]
    return {"solver": stype, "solved": bool(solved), "score": {k: float(v) for k, v in score.items()},
            "published_score": ref, "published_processing_time_s": ref_t, "wall_s": wall,
            "allocations": c, "steps": steps,
            "matches": {k: abs(float(score[k]) - ref[k]) <= 1e-6 * max(1.0, abs(ref[k])) for k in ref}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--step-seconds", type=float, default=60.0)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="")
    ap.add_argument("--solvers", default="NeptuneMinDelay,NeptuneMinDelayAndUtilization,NeptuneMinUtilization")
    a = ap.parse_args()
    out = []
    for st in a.solvers.split(","):
        r = run(st, a.step_seconds, a.batch)
        print(json.dumps({k: r[k] for k in ("solver", "score", "published_score", "wall_s", "matches")}), flush=True)
        for k, v in r["steps"].items():
            print("   ", k, json.dumps(v), flush=True)
        out.append(r)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
