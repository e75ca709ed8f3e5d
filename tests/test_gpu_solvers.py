"""GPU twin of tests/test_bnb_cpu.py: the drop-in NEPTUNE solver classes (core/solvers) run the
two-step flow on the MI355X engine — batched PDHG node LPs, warm-started from their parents
(core/engine/bnb.py) — and must reproduce the reference flow's responses recorded in the golden
fixtures: both scores, and — where the reference optimum is unique — the whole wire format
(allocations; routing sources, and for functions with one open destination — where the routing is
forced — every destination and rounded value)."""
import pytest

from golden_util import golden, payload

pytestmark = pytest.mark.gpu
G = golden()
CASES = ["payload", "testpy", "syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization", "syn_4x3_s0_r0.5_NeptuneMinDelay",
         "syn_4x3_s0_r0.5_NeptuneMinUtilization", "syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization",
         "syn_6x4_s1_r0.3_NeptuneMinDelay", "syn_6x4_s1_r0.3_NeptuneMinUtilization",
         "syn_8x4_s2_r0.1_NeptuneMinDelayAndUtilization", "sim0_NeptuneMinDelay", "sim3_NeptuneMinDelayAndUtilization",
         "sim2_NeptuneMinUtilization", "sim4_NeptuneMinUtilization"]


def _close(a, b, tol=1e-6):
    return abs(a - b) <= tol * max(1.0, abs(b))


@pytest.mark.parametrize("name", CASES)
def test_solver_flow_on_gpu(name):
    import core.solvers as S
    from core.utils import data_to_solver_input
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    solver.load_data(data)
    solver.solve()
    x, c = solver.results()
    score = solver.score()
    ref = G[name]["response"]
    assert _close(score["step1"], ref["score"]["step1"]), (score, ref["score"])
    assert _close(score["step2"], ref["score"]["step2"]), (score, ref["score"])
    done = [m for m in G[name]["models"] if m["status"] == 0]
    if done and done[-1].get("mip_tied") is False:
        # unique optimum: the whole wire format — allocations, and every routing entry's source,
        # function, destination and rounded value (output.py:23-39) within 1e-3
        assert c == ref["cpu_allocations"]
        rr = ref["cpu_routing_rules"]
        assert set(x) == set(rr)
        for src, fns in rr.items():
            assert set(x[src]) == set(fns), (src, x[src], fns)
            for fn, dsts in fns.items():
                if len(ref["cpu_allocations"].get(fn, {})) != 1:
                    continue     # several open destinations: the routing may have tied optima
                assert set(x[src][fn]) == set(dsts), (src, fn, x[src][fn], dsts)
                for dst, val in dsts.items():
                    assert abs(x[src][fn][dst] - val) <= 1e-3, (src, fn, dst, x[src][fn][dst], val)


@pytest.mark.parametrize("name", CASES)
def test_solver_step1_search_is_optimal(name):
    """The step-1 search itself ends OPTIMAL (not LIMIT with a matching score) wherever the reference's
    recorded step-1 MIP has an optimum — SCIP proves these small instances at once (round-3 VERDICT: testpy's
    3x2 step 1 ended LIMIT)."""
    import core.solvers as S
    from core.utils import data_to_solver_input
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    step1 = getattr(solver, "step1", None)
    if step1 is None or not hasattr(step1, "branch_and_bound") or G[name]["models"][0]["status"] != 0:
        pytest.skip("no NEPTUNE step 1 / no recorded step-1 optimum")
    step1.load_data(data)
    step1.solve()
    r = step1.result
    print(name, r.status, r.objective, r.bound, r.nodes, r.lps, r.as_dict()["lp_status_kind"])
    assert r.status == "OPTIMAL", (r.status, r.objective, r.bound)
    assert _close(r.objective, G[name]["models"][0]["mip_objective"])
