#!/usr/bin/env python3
"""Golden responses of the reference's EF-TTC solvers (build container only; writes
tests/golden/efttc.json).

The reference's own classes run unmodified (imported exactly as tools/gen_golden.py does, with the
probe-only pywraplp / hurry stand-ins of tools/refshim; the NEPTUNE step-2 MIPs are solved by
HiGHS through the recording stand-in):
  * EfttcMinDelay / EfttcMinUtilization / EfttcMinDelayAndUtilization  (core/solvers/efttc/efttc.py:29-48)
  * NeptuneWithEFTTC{MinDelay, MinUtilization, MinDelayAndUtilization}  (core/solvers/neptune/neptune.py:68-93)
on the committed inputs (tests/golden/inputs), the second family on the small ones only.  Recorded:
the REST response (routing, allocations, score) and the EF-TTC step-1 placement (c, n, score).

  python3 tools/gen_efttc_golden.py
"""
import contextlib
import io
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (sets up the reference import with the stand-ins)

REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "efttc.json")
EFTTC = ("EfttcMinDelay", "EfttcMinUtilization", "EfttcMinDelayAndUtilization")
WITH = ("NeptuneWithEFTTCMinDelay", "NeptuneWithEFTTCMinUtilization", "NeptuneWithEFTTCMinDelayAndUtilization")
SMALL = ("payload", "testpy", "sim0", "sim1", "sim2", "sim3", "sim4", "syn_4x3", "syn_6x4", "syn_8x4_s2")


def step1_placement(solver):
    """c, n of the EF-TTC step 1 (efttc_step1.py) after solve()."""
    s1 = solver.step1
    F, N = len(s1.data.functions), len(s1.data.nodes)
    c = [[1 if s1.c[(f, j)]["val"] else 0 for j in range(N)] for f in range(F)]
    n = [1 if s1.n[j]["val"] else 0 for j in range(N)]
    return {"c": c, "n": n}


def run(payload, stype):
    p = json.loads(json.dumps(payload))
    p["solver"] = dict(p.get("solver", {}))
    p["solver"]["type"] = stype
    G.pywraplp.Solver.RECORD = []
    G.pywraplp.Solver.RELAX = False
    buf = io.StringIO()
    t0 = time.time()
    with contextlib.redirect_stdout(buf):
        G.check_input(p)
        cls = getattr(G.RS, stype)
        s = cls(**p["solver"].get("args", {}))
        data = G.data_to_solver_input(p, with_db=p.get("with_db", True), workload_coeff=p.get("workload_coeff", 1))
        s.load_data(data)
        solved = s.solve()
        x, c = s.results()
        score = s.score()
    G.pywraplp.Solver.RECORD = None
    return {"response": {"cpu_routing_rules": x, "cpu_allocations": c, "score": score}, "solved": bool(solved),
            "step1": step1_placement(s), "elapsed_s": round(time.time() - t0, 3)}


def main():
    inputs = os.path.join(REPO, "tests", "golden", "inputs")
    out = {}
    for fn in sorted(os.listdir(inputs)):
        name = fn[:-5]
        with open(os.path.join(inputs, fn)) as fh:
            payload = json.load(fh)
        small = any(name.startswith(k) for k in SMALL)
        types = EFTTC + (WITH if small else ())
        for t in types:
            key = f"{name}|{t}"
            try:
                out[key] = run(payload, t)
                print(key, out[key]["response"]["score"], out[key]["elapsed_s"], "s", flush=True)
            except Exception as e:  # the reference raising is a recorded outcome too
                out[key] = {"error": f"{type(e).__name__}: {e}"}
                print(key, "ERROR", out[key]["error"], flush=True)
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=None, separators=(",", ":"))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
