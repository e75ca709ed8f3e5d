"""EF-TTC (core/solvers/efttc) against the reference's own outputs (tests/golden/efttc.json, recorded
by tools/gen_efttc_golden.py from the unmodified reference classes):

* Efttc{MinDelay, MinUtilization, MinDelayAndUtilization}: the whole REST response — routing (sources,
  destinations and rounded values), allocations and both scores — equals the reference's, and inputs
  on which the reference raises raise the same exception type;
* NeptuneWithEFTTC*: the EF-TTC step-1 placement (c, n) and score equal the reference's, and the full
  two-step flow (step 2 = the NEPTUNE MIP, here with the CPU oracle as node-LP backend, as in
  tests/test_bnb_cpu.py) reproduces both scores.  The GPU twin is tests/test_gpu_efttc.py."""
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN

with open(os.path.join(GOLDEN, "efttc.json")) as fh:
    E = json.load(fh)
EFTTC = sorted(k for k in E if k.split("|")[1].startswith("Efttc"))
WITH = sorted(k for k in E if k.split("|")[1].startswith("NeptuneWithEFTTC") and "error" not in E[k])


def _payload(key):
    name, stype = key.split("|")
    with open(os.path.join(GOLDEN, "inputs", name + ".json")) as fh:
        p = json.load(fh)
    p["solver"] = dict(p.get("solver", {}))
    p["solver"]["type"] = stype
    return p


def _data(p):
    from core.utils import data_to_solver_input
    return data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)


def _close(a, b, tol=1e-9):
    return abs(float(a) - float(b)) <= tol * max(1.0, abs(float(b)))


@pytest.mark.parametrize("key", EFTTC)
def test_efttc_response_matches_reference(key):
    import core.solvers as S
    p = _payload(key)
    ref = E[key]
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    data = _data(p)
    solver.load_data(data)
    if "error" in ref:
        with pytest.raises(Exception) as ei:
            solver.solve()
        assert ref["error"].startswith(type(ei.value).__name__), (ref["error"], repr(ei.value))
        return
    solver.solve()
    x, c = solver.results()
    score = solver.score()
    r = ref["response"]
    assert _close(score["step1"], r["score"]["step1"]) and score["step2"] == r["score"]["step2"], (score, r["score"])
    assert c == r["cpu_allocations"]
    assert x == r["cpu_routing_rules"]


@pytest.mark.parametrize("key", WITH)
def test_neptune_with_efttc_flow(key, monkeypatch):
    import core.solvers as S
    from core.solvers.neptune import neptune_step
    from oracle_lp import OracleLP
    monkeypatch.setattr(neptune_step, "make_lp",
                        lambda data, variant, step, max_batch, **kw: OracleLP(data, variant, step=step,
                                                                              max_batch=max_batch, **kw))
    p = _payload(key)
    ref = E[key]
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    data = _data(p)
    solver.load_data(data)
    solver.solve()
    s1 = solver.step1
    assert np.array_equal(s1.c.astype(int), np.array(ref["step1"]["c"])), "EF-TTC step-1 allocations differ"
    assert np.array_equal(s1.n.astype(int), np.array(ref["step1"]["n"])), "EF-TTC step-1 nodes differ"
    score = solver.score()
    r = ref["response"]["score"]
    assert _close(score["step1"], r["step1"]), (score, r)
    assert _close(score["step2"], r["step2"], 1e-6), (score, r)
