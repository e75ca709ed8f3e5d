"""CPU suite: the C-ABI engine library (neptune-mip_amd/lib/libneptune_lp.so) loads and exports every
entry point include/neptune_lp.h declares, and its host-only model build (nep_debug_build: zero-workload
aggregation, Ruiz + Pock-Chambolle scaling, row norms, power-iteration step size) equals the test-only
numpy mirror tests/ref_pdhg.py.  No device calls: nothing here needs a GPU."""
import os
import re

import numpy as np
import pytest

from gpu_cases import build_args, lp_cases

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "neptune_lp.h")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|void \*|void|const char \*)\s*(nep_\w+)\(", text, re.M)))


def test_header_declares_exactly_the_binding_exports():
    from core.engine import lp
    assert declared() == sorted(lp.EXPORTS)


def test_library_exports_every_declared_symbol():
    from core.engine import lp
    lib = lp.load_library()
    missing = [s for s in declared() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.nep_api_version() == lp.API_VERSION


def test_bad_arguments_fail_loudly():
    """Errors come back as return codes + nep_last_error, raised as EngineUnavailable (no device work)."""
    from core.engine import lp
    from golden_util import payload
    from core.utils import data_to_solver_input
    data = data_to_solver_input(payload("payload"), with_db=False)
    with pytest.raises(lp.EngineUnavailable, match="bad variant"):
        lp.debug_build(data, 7)


def test_api12_entries_reject_null_model():
    """The round-6 entry points (nep_lp_submit_ex, nep_lp_copy_states, nep_lp_get_flows_solutions,
    nep_debug_sparse_rows) return NEP_ERR_ARG with a message for a null model, before any device work."""
    from core.engine import lp
    lib = lp.load_library()
    for name, args in (("nep_lp_submit_ex", (None, 1, None, None, None, None, None, None, None)),
                       ("nep_lp_copy_states", (None, 1, None, None)),
                       ("nep_lp_get_flows_solutions", (None, 1, None, None, None)),
                       ("nep_debug_sparse_rows", (None, 0, None, None))):
        assert getattr(lib, name)(*args) == -1, name
        assert lib.nep_last_error(), name


CASES = lp_cases(max_vars=2000)


@pytest.mark.parametrize("name,k", CASES)
def test_host_build_matches_mirror(name, k):
    from core.engine.lp import debug_build
    from ref_pdhg import RefModel
    data, variant, step, kw = build_args(name, k)
    got = debug_build(data, variant, step=step, **kw)
    ref = RefModel(data, variant, step=step, **kw)
    assert (got["R"], got["T"], got["n_int"], got["n_dual"]) == (ref.R, ref.F, ref.n_int, ref.n_dual)
    np.testing.assert_allclose(got["rho"], ref.rho, rtol=1e-10)
    np.testing.assert_allclose(got["gam"], ref.gam, rtol=1e-10)
    np.testing.assert_allclose(got["rownorm"], ref.rownorm, rtol=1e-12)
    # power iteration from different random starts (60 steps each): the same operator norm within 1 % (the
    # step size eta = 0.95 / ||K~|| keeps 5 % of headroom; the reduced step-2 operator's top singular values
    # are close, so 60 steps agree to ~5e-3 there)
    assert abs(got["eta"] / ref.eta - 1.0) < 1e-2


@pytest.mark.parametrize("name,k", CASES)
def test_node_presolve_incremental_equals_full(name, k):
    """nep_lp_submit presolves a node as a sparse change of the model's base box (presolve_node);
    it must decide feasibility and produce the node box exactly as the from-scratch presolve does."""
    from core.engine.lp import debug_build, debug_presolve
    data, variant, step, kw = build_args(name, k)
    n_int = debug_build(data, variant, step=step, **kw)["n_int"]
    N, F = len(data.nodes), len(data.functions)
    rng = np.random.default_rng(k + 17)
    nodes = 24
    lb = np.full((nodes, n_int), -np.inf)
    ub = np.full((nodes, n_int), np.inf)
    for b in range(nodes):
        kind = b % 4
        if kind == 0:                      # a few 0/1 fixings anywhere (crossed bounds included)
            idx = rng.choice(n_int, size=min(n_int, 3), replace=False)
            val = rng.integers(0, 2, size=idx.size).astype(float)
            lb[b, idx] = val
            ub[b, idx] = val
        elif kind == 1:                    # placements of one function closed but one
            f = int(rng.integers(F))
            ub[b, f * N:(f + 1) * N] = 0.0
            ub[b, f * N + int(rng.integers(N))] = np.inf
        elif kind == 2:                    # every placement of one function closed: infeasible (C4)
            f = int(rng.integers(F))
            ub[b, f * N:(f + 1) * N] = 0.0
        else:                              # a node closed (n_j = 0 when the model has n) + a placement forced there
            j = int(rng.integers(N))
            ub[b, n_int - N + j] = 0.0
            lb[b, int(rng.integers(F)) * N + j] = 1.0
    ok_f, ok_n, box_f, box_n = debug_presolve(data, variant, lb, ub, step=step, **kw)
    np.testing.assert_array_equal(ok_f, ok_n)
    assert not ok_f[2::4].any()
    for b in np.nonzero(ok_f)[0]:
        np.testing.assert_array_equal(box_f[b], box_n[b])


def test_parallel_node_presolve_equals_full():
    """Above ~8k integer variables nep_lp_submit presolves a batch's nodes on several host threads
    (nep_host.cpp presolve_batch; rounding leaves fix every c and n and take the dense row re-test): each
    node must still decide feasibility and produce the box the from-scratch presolve does."""
    from core.engine.heuristics import capacity_greedy
    from core.engine.lp import debug_build, debug_presolve
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F = 128, 64
    data = data_to_solver_input(synthetic_payload(N, F, seed=3), with_db=False)
    n_int = debug_build(data, "MinDelayAndUtilization", step=1, alpha=0.5)["n_int"]
    assert n_int >= 8192
    rng = np.random.default_rng(5)
    d = data
    leaves = capacity_greedy(d.workload_matrix, d.node_delay_matrix, d.core_per_req_matrix,
                             np.reshape(d.node_cores_matrix, N), np.reshape(d.function_memory_matrix, F),
                             np.reshape(d.node_memory_matrix, N), np.asarray(d.node_cores_matrix, float).reshape(N))
    B = 12
    lb = np.full((B, n_int), -np.inf)
    ub = np.full((B, n_int), np.inf)
    for b in range(B):
        if b % 3 == 0:                     # a rounding leaf: every c and n fixed (the capacity greedy's)
            c, n = leaves[(b // 3) % len(leaves)][:2]
            c, n = np.asarray(c, float).reshape(-1), np.asarray(n, float).copy()
            if b % 6 == 0:                 # (an open placement on a closed node: infeasible)
                n[int(np.nonzero(c.reshape(F, N).max(0))[0][0])] = 0.0
            lb[b, :F * N] = ub[b, :F * N] = c
            lb[b, F * N:] = ub[b, F * N:] = n
        elif b % 3 == 1:                   # a branching node: a few fixings
            idx = rng.choice(n_int, 6, replace=False)
            lb[b, idx] = ub[b, idx] = rng.integers(0, 2, idx.size)
        else:                              # every placement of one function closed: infeasible (C4)
            f = int(rng.integers(F))
            ub[b, f * N:(f + 1) * N] = 0.0
    ok_f, ok_n, box_f, box_n = debug_presolve(data, "MinDelayAndUtilization", lb, ub, step=1, alpha=0.5)
    np.testing.assert_array_equal(ok_f, ok_n)
    assert not ok_f[2::3].any() and not ok_f[0::6].any() and ok_n[1] and ok_n[3::6].all()
    for b in np.nonzero(ok_f)[0]:
        np.testing.assert_array_equal(box_f[b], box_n[b])


def test_request_unknown_solver_type_raises():
    """core.request resolves solver.type through the SOLVERS whitelist (the reference: eval, main.py:44);
    an unknown type raises before any engine call (the reference's server answers HTTP 500)."""
    import copy
    import pytest
    from core.request import solve_request
    from golden_util import payload
    p = copy.deepcopy(payload("payload"))
    p["solver"] = {"type": "NotASolver"}
    with pytest.raises(KeyError):
        solve_request(p)


@pytest.mark.parametrize("name,k", CASES[:4])
def test_inline_reflection_equals_tracked_activity(name, k):
    """x_pass forms the C1/C2/D1/D2 reflected activities K(2ŵ - w) from the primal points instead of
    tracking K w (kz / kza): the same PDHG operator, so the mirror reaches the same answer either way."""
    from ref_pdhg import RefModel, solve
    data, variant, step, kw = build_args(name, k)
    ref = RefModel(data, variant, step=step, **kw)
    a = solve(ref, tol=1e-6, max_iters=20000, check_every=16)
    b = solve(ref, tol=1e-6, max_iters=20000, check_every=16, inline_reflect=True)
    assert a["status"] == b["status"]
    if a["status"] == 0:
        assert abs(a["obj"] - b["obj"]) <= 1e-5 * max(1.0, abs(a["obj"]))
        assert abs(a["iters"] - b["iters"]) <= 0.1 * a["iters"] + 16


def test_facility_relaxation_build():
    """nep_debug_build of the B&B's facility relaxation (NEP_RELAX_FACILITY, API 7): its dual rows are C3, C5
    and c[f,j] <= n[j] (2N + FN; the x <= c rows are per routing entry, outside the dual vector), the integer
    vector is step 1's (c, n), and it exists only for step-1 models with n (MinUtilization / MDU)."""
    from core.engine.lp import EngineUnavailable, RELAX_FACILITY, STEP2_CREATE, debug_build
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F = 16, 8
    data = data_to_solver_input(synthetic_payload(N, F, seed=0), with_db=False)
    ref = debug_build(data, "MinDelayAndUtilization")
    got = debug_build(data, "MinDelayAndUtilization", relaxation=RELAX_FACILITY)
    assert got["n_dual"] == 2 * N + F * N and got["n_int"] == F * N + N == ref["n_int"]
    assert got["R"] == ref["R"] and 0.0 < got["eta"] < float("inf")
    assert np.all(np.isfinite(got["rho"])) and np.all(got["rho"] > 0) and np.all(got["gam"] > 0)
    for variant, step in (("MinDelay", 1), ("MinDelayAndUtilization", STEP2_CREATE)):
        with pytest.raises(EngineUnavailable):
            debug_build(data, variant, step=step, relaxation=RELAX_FACILITY, max_score=1.0)


def test_presolve_cpu_cover_proves_overloaded_leaf_infeasible():
    """The node presolve's CPU cover test (nep_host.cpp cpu_cover_ok): testpy's step-1 rounding leaf that opens
    node 0 only (c[0,0] = c[1,0] = n[0] = 1, everything else 0) overloads node 0's CPU — HiGHS finds the box
    infeasible (tools/probes/leaf_limit_probe.py) and PDHG could only stall on it (round-4 GPU suite: testpy's step 1
    ended LIMIT).  Both the from-scratch and the sparse-change presolve must reject it, and the leaf that
    also opens node 1 must pass."""
    import numpy as np
    from golden_util import payload
    from core.engine.lp import debug_presolve
    from core.utils import data_to_solver_input
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve
    p = payload("testpy")
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    N, F = len(data.nodes), len(data.functions)
    variant = {"NeptuneMinDelayAndUtilization": "MinDelayAndUtilization", "NeptuneMinUtilization": "MinUtilization",
               "NeptuneMinDelay": "MinDelay"}[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    n_int = F * N + N
    lb = np.zeros((2, n_int))
    ub = np.zeros((2, n_int))
    for b, opened in enumerate(([0, 3, 6], [0, 3, 4, 6, 7])):
        lb[b, opened] = ub[b, opened] = 1.0
    ok_full, ok_node, _, _ = debug_presolve(data, variant, lb, ub, step=1, alpha=alpha)
    ref = build_model(oracle_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False), variant, step=1,
                      alpha=alpha)
    nx = N * N * F
    for b in range(2):
        rl, ru = ref["lb"].copy(), ref["ub"].copy()
        rl[nx:], ru[nx:] = lb[b], ub[b]
        st, _, _ = solve(ref, relax=True, lb=rl, ub=ru)
        assert bool(ok_full[b]) == bool(ok_node[b]) == (st == 0), (b, ok_full[b], ok_node[b], st)
    assert not ok_full[0]
