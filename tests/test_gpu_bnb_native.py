"""The native tree search (csrc/nep_bnb.cpp, nep_bnb_*) against core/engine/bnb.py's Python
loop: on the golden step-1 instances both searches end OPTIMAL at the recorded MIP with the same tree (nodes,
LPs — bnb.py's decision order and tie-breaks, the same engine calls), and on the 64x32 / 256x128 synthetic
instances the native loop spends less host time per node LP (everything outside the device waits of nep_lp_advance)
than the Python loop (profiles/r05/native)."""
import math

import pytest

from golden_util import golden, payload

pytestmark = pytest.mark.gpu
G = golden()
CASES = ["payload", "testpy", "syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization", "syn_4x3_s0_r0.5_NeptuneMinDelay",
         "syn_4x3_s0_r0.5_NeptuneMinUtilization", "syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization",
         "syn_8x4_s2_r0.1_NeptuneMinDelayAndUtilization", "sim0_NeptuneMinDelay", "sim3_NeptuneMinDelayAndUtilization",
         "sim2_NeptuneMinUtilization"]


def _search(step1, data, native, **kw):
    from core.solvers.neptune.neptune_step import make_lp
    model = make_lp(data, step1.VARIANT, step1.step_id(), step1.batch + 2, **step1.model_kwargs())
    bmodel = None
    try:
        bmodel = step1.bound_model(data, step1.batch + 1)
        return step1.branch_and_bound(model, bmodel, native=native, **kw).solve()
    finally:
        model.close()
        if bmodel is not None:
            bmodel.close()


@pytest.mark.parametrize("name", CASES)
def test_native_search_matches_python(name):
    import core.solvers as S
    from core.utils import data_to_solver_input
    if name not in G:
        pytest.skip("no golden")
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    step1 = getattr(solver, "step1", None)
    if step1 is None or not hasattr(step1, "branch_and_bound") or G[name]["models"][0]["status"] != 0:
        pytest.skip("no NEPTUNE step 1 / no recorded step-1 optimum")
    step1.load_data(data)
    # (the loops are compared on the flow rule, the one the Python loop implements; the product's reliability
    # branching runs on the native tree only and is checked by tests/test_gpu_solvers.py)
    rp = _search(step1, data, False, branching=0)
    rn = _search(step1, data, True, branching=0)
    print(name, "python", rp.status, rp.objective, rp.nodes, rp.lps, "| native", rn.status, rn.objective, rn.nodes,
          rn.lps)
    assert rn.native and not rp.native
    assert rn.status == rp.status == "OPTIMAL"
    ref = G[name]["models"][0]["mip_objective"]
    assert abs(rn.objective - ref) <= 1e-6 * max(1.0, abs(ref))
    assert abs(rn.objective - rp.objective) <= 1e-9 * max(1.0, abs(rp.objective))
    assert (rn.nodes, rn.lps, rn.leaves) == (rp.nodes, rp.lps, rp.leaves)


@pytest.mark.parametrize("n,f,seconds", [(64, 32, 10.0), (256, 128, 20.0)])
def test_native_search_host_share(n, f, seconds):
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    data = data_to_solver_input(synthetic_payload(n, f, seed=0), with_db=False)
    out = {}
    for native in (False, True):
        st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6, lp_max_iters=4096)
        st1.load_data(data)
        r = _search(st1, data, native, time_limit=seconds)
        tm = r.timing
        wall = r.seconds
        host = 1.0 - tm["advance"] / wall
        out[native] = (host, r.nodes, r.lps, r.objective, r.bound, (wall - tm["advance"]) / max(1, r.lps))
        print(f"{n}x{f} {'native' if native else 'python'}: host {host:.3f} of {wall:.1f} s, nodes {r.nodes}, lps {r.lps}, "
              f"incumbent {r.objective}, bound {r.bound}, timing {dict((k, round(v, 2)) for k, v in tm.items())}")
        assert r.objective is not None and math.isfinite(r.bound) and r.bound <= r.objective + 1e-9
    # host seconds per node LP: at 64x32, where the per-LP Python work was the host's time, the native loop's is
    # below the Python loop's (at 256x128 both are the native submit / rounding / device reads: equal within noise).
    # The host SHARE depends on how fast the LPs converge (DESIGN.md §7 "Native tree search"): 0.242-0.253 measured
    # at 64x32 over four boxes of round 6 (the round-4 target 0.25; round 5: 0.29) — the bar keeps box-to-box slack
    print(f"host seconds per LP: python {out[False][5] * 1e6:.0f} us, native {out[True][5] * 1e6:.0f} us")
    assert out[True][0] < 0.30
    if n <= 64:
        assert out[True][5] < out[False][5]


FLOW_CASES = ["payload", "testpy", "syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization", "syn_6x4_s1_r0.3_NeptuneMinDelay",
              "syn_8x4_s2_r0.1_NeptuneMinDelayAndUtilization", "sim3_NeptuneMinDelayAndUtilization"]


@pytest.mark.parametrize("name", FLOW_CASES)
def test_native_step2_matches_python(name, monkeypatch):
    """Step 2 on the native tree (the integer bound in C++, node relocation on NEP_BNB_INCUMBENT events): the whole
    NEPTUNE flow gives the same step-1 / step-2 scores as with the Python loop (NEP_BNB_PYTHON=1), both equal to the
    reference's recorded ones."""
    import core.solvers as S
    from core.utils import data_to_solver_input
    if name not in G:
        pytest.skip("no golden")
    p = payload(name)
    scores, native = {}, {}
    monkeypatch.setenv("NEP_BNB_STEP2", "1")
    for py in ("1", "0"):
        monkeypatch.setenv("NEP_BNB_PYTHON", py)
        data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
        solver = S.SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
        if not hasattr(solver, "step2_delete"):
            pytest.skip("not a NEPTUNE flow")
        solver.load_data(data)
        solver.solve()
        scores[py] = solver.score()
        steps = [s for s in (solver.step2_delete, solver.step2_create) if getattr(s, "result", None) is not None]
        native[py] = [bool(getattr(s.result, "native", False)) for s in steps]
    print(name, scores, native)
    ref = G[name]["response"]["score"]
    for py in ("1", "0"):
        assert abs(scores[py]["step1"] - ref["step1"]) <= 1e-6 * max(1.0, abs(ref["step1"]))
        assert abs(scores[py]["step2"] - ref["step2"]) <= 1e-6 * max(1.0, abs(ref["step2"]))
    assert not any(native["1"]) and native["0"] and all(native["0"])
