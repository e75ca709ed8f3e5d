"""The product's branch-and-bound (core/engine/bnb.py) and two-step orchestration (core/solvers/neptune)
run on CPU with the ORACLE as node-LP backend (tests/oracle_lp.py): they must reproduce the MIP
optima HiGHS found on the reference's own recorded models, and the responses of the reference
flow (scores; placements where the optimum is unique).  The GPU twin is tests/test_gpu_solvers.py."""
import numpy as np
import pytest

from golden_util import golden, model, payload
from gpu_cases import VARIANT
from oracle_lp import OracleLP

G = golden()
SMALL = [(name, k) for name, v in G.items() if "models" in v
         for k, m in enumerate(v["models"]) if m["n_vars"] <= 400]
FLOW = [name for name, v in G.items() if "response" in v and max(m["n_vars"] for m in v["models"]) <= 400]


def _data(name):
    from core.utils import data_to_solver_input
    p = payload(name)
    return p, data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)


def _close(a, b):
    return abs(a - b) <= 1e-6 * max(1.0, abs(b))


@pytest.mark.parametrize("name,k", SMALL)
def test_bnb_matches_recorded_mip(name, k):
    from core.engine.bnb import INFEASIBLE, OPTIMAL, BranchAndBound
    p, data = _data(name)
    rec = G[name]["models"][k]
    variant = VARIANT[p["solver"]["type"]]
    args = p["solver"].get("args", {})
    kw = dict(alpha=args.get("alpha", 0.5), soften_step1_sol=args.get("soften_step1_sol", 1.3))
    step = 1
    if k > 0:
        N, F = len(data.nodes), len(data.functions)
        m1 = model(name, 0)
        data.prev_x = m1["mip_x"][:N * N * F].reshape(F, N, N).transpose(1, 0, 2)
        kw["max_score"] = float(m1["mip_objective"])
        step = 2 if rec["mode"] == "step2_delete" else 3
    lp = OracleLP(data, variant, step=step, max_batch=17, **kw)    # 2 x batch + root: warm-start slots
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=20000).solve()
    if res.lps > 1:
        assert getattr(lp, "copies", 0) > 0, "warm-start slot hand-offs never ran"
    if rec["status"] == 0:
        assert res.status == OPTIMAL, res.as_dict()
        assert _close(res.objective, rec["mip_objective"]), (res.objective, rec["mip_objective"])
    else:
        assert res.status == INFEASIBLE, res.as_dict()


@pytest.mark.parametrize("name", FLOW)
def test_solver_flow_matches_reference(name, monkeypatch):
    import core.solvers as S
    from core.solvers.neptune import neptune_step
    monkeypatch.setattr(neptune_step, "make_lp",
                        lambda data, variant, step, max_batch, **kw: OracleLP(data, variant, step=step,
                                                                              max_batch=max_batch, **kw))
    p, data = _data(name)
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
        assert c == ref["cpu_allocations"]
        assert set(x) == set(ref["cpu_routing_rules"])


STEP1 = [(name, k) for name, k in SMALL if k == 0][:10]


@pytest.mark.parametrize("name,k", STEP1)
def test_bnb_with_bound_converged_nodes(name, k):
    """Branching nodes that end NEP_LP_BOUND (bound converged, primal not certified: nep_lp_opts.bound_res)
    branch on their bound like certified ones; leaves still need certificates.  The streaming fake engine
    returns LP_BOUND for every LP submitted with bound_res > 0: the search must still reach the recorded
    MIP optimum, and only leaves may be counted certified."""
    from core.engine.bnb import INFEASIBLE, OPTIMAL, BranchAndBound
    from oracle_lp import StreamingOracleLP
    p, data = _data(name)
    rec = G[name]["models"][k]
    variant = VARIANT[p["solver"]["type"]]
    args = p["solver"].get("args", {})
    lp = StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=args.get("alpha", 0.5))
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=20000, node_bound_res=1e-2).solve()
    if rec["status"] == 0:
        assert res.status == OPTIMAL, res.as_dict()
        assert _close(res.objective, rec["mip_objective"]), (res.objective, rec["mip_objective"])
    else:
        assert res.status == INFEASIBLE, res.as_dict()
    assert res.lp_status_kind["node"]["certified"] <= 1      # (the root alone may certify)
    assert res.lp_status["bound"] == res.lp_status_kind["node"]["bound"]


STEP1_N = [(n, k) for n, k in SMALL if k == 0 and VARIANT[payload(n)["solver"]["type"]] != "MinDelay"]


@pytest.mark.parametrize("name,k", STEP1_N)
def test_bnb_two_models_matches_recorded_mip(name, k):
    """Round 4: the branching nodes bounded by the facility relaxation (a second model,
    oracle/formulation.py facility_relaxation: x <= c, c <= n in place of the big-M pairs), the leaves solved
    on the reference model: the search still reaches the MIP optimum HiGHS found on the reference's own
    recorded model (the relaxation is valid for every integral placement, so no optimum is cut off), with
    streaming out-of-order finishes on both models."""
    from core.engine.bnb import INFEASIBLE, OPTIMAL, BranchAndBound
    from oracle_lp import StreamingOracleLP
    p, data = _data(name)
    rec = G[name]["models"][k]
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    lp = StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=alpha)
    blp = StreamingOracleLP(data, variant, step=1, max_batch=9, alpha=alpha, relaxation=1)
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=20000, bound_lp=blp).solve()
    if rec["status"] == 0:
        assert res.status == OPTIMAL, res.as_dict()
        assert _close(res.objective, rec["mip_objective"]), (res.objective, rec["mip_objective"])
    else:
        assert res.status == INFEASIBLE, res.as_dict()
    assert res.lp_status_kind["refroot"]["certified"] + res.lp_status_kind["refroot"]["cutoff"] <= 1
    assert res.routing_warm == getattr(lp, "routing_copies", 0)


@pytest.mark.parametrize("name,k", STEP1_N[:8])
def test_bnb_primal_heuristic_keeps_optimum(name, k):
    """The capacity-greedy primal heuristic (core/engine/heuristics.py, NeptuneStepBase.primal_heuristic) hooked
    into the two-model search: its leaves are feasible for the reference rows (every one the leaf LP solves
    is an integral placement of the reference model), so the search still ends at the recorded MIP optimum."""
    from core.engine.bnb import INFEASIBLE, OPTIMAL, BranchAndBound
    from core.solvers import SOLVERS
    from oracle_lp import StreamingOracleLP
    p, data = _data(name)
    rec = G[name]["models"][k]
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    solver = SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    step1 = solver.step1 if hasattr(solver, "step1") else solver
    step1.load_data(data)
    lp = StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=alpha)
    blp = StreamingOracleLP(data, variant, step=1, max_batch=9, alpha=alpha, relaxation=1)
    primal = step1.primal_heuristic(lp.layout(), lp.row_map())
    assert primal is not None
    calls, sols = [], []

    def hook(*a):
        out = primal(*a)
        calls.append(1)
        sols.extend(item[2] for item in out if item[2] is not None)
        return out
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=20000, bound_lp=blp, primal_every=4, primal=hook).solve()
    assert calls
    for sol in sols:   # every checked greedy point is feasible: its objective is >= the MIP optimum
        assert sol["objective"] >= rec["mip_objective"] - 1e-6 * max(1.0, abs(rec["mip_objective"]))
    if rec["status"] == 0:
        assert res.status == OPTIMAL, res.as_dict()
        assert _close(res.objective, rec["mip_objective"]), (res.objective, rec["mip_objective"])
    else:
        assert res.status == INFEASIBLE, res.as_dict()


@pytest.mark.parametrize("name,k", STEP1_N[:8])
def test_heuristic_incumbent_is_feasible_reference_point(name, k):
    """A checked capacity-greedy point taken as the incumbent (BranchAndBound._heuristic_incumbent) before any
    leaf LP: stopped right after the root (node_limit=1), the search returns it — and its (z, routing) is a
    feasible point of the reference formulation (oracle/formulation.py rows, fp64) whose objective is the
    returned one."""
    from core.engine.bnb import BranchAndBound
    from core.solvers import SOLVERS
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle_lp import StreamingOracleLP
    p, data = _data(name)
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    solver = SOLVERS[p["solver"]["type"]](**p["solver"].get("args", {}))
    step1 = solver.step1 if hasattr(solver, "step1") else solver
    step1.load_data(data)
    lp = StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=alpha)
    blp = StreamingOracleLP(data, variant, step=1, max_batch=9, alpha=alpha, relaxation=1)
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=1, bound_lp=blp, polish_tol=0,
                         primal=step1.primal_heuristic(lp.layout(), lp.row_map())).solve()
    if not res.heuristic_incumbents:
        pytest.skip("the greedy found no checked point at the root of this instance")
    N, F = len(data.nodes), len(data.functions)
    m = build_model(oracle_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False), variant, step=1,
                    alpha=alpha)
    x = np.zeros((F, N, N))
    i, f, j, v = res.x.entries()
    x[f, i, j] = v
    full = np.concatenate([x.ravel(), np.asarray(res.z, np.float64)])
    act = m["A"] @ full
    assert (act <= m["hi"] + 1e-6).all() and (act >= m["lo"] - 1e-6).all()
    assert (full >= m["lb"] - 1e-12).all() and (full <= m["ub"] + 1e-12).all()
    assert abs(float(m["c"] @ full) - res.objective) <= 1e-9 * max(1.0, abs(res.objective))



def test_two_model_leaves_take_routing_warm_starts():
    """Leaves of the two-model search start from their branching node's routing (nep_lp_copy_routing) when
    that node's bound-model slot still holds it: across the step-1 goldens some do, and every hand-off reads a
    slot the bound model solved (the oracle stub asserts it)."""
    from core.engine.bnb import BranchAndBound
    from oracle_lp import StreamingOracleLP
    total = 0
    for name, k in STEP1_N[:6]:
        p, data = _data(name)
        variant = VARIANT[p["solver"]["type"]]
        alpha = p["solver"].get("args", {}).get("alpha", 0.5)
        lp = StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=alpha)
        blp = StreamingOracleLP(data, variant, step=1, max_batch=9, alpha=alpha, relaxation=1)
        res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                             batch=8, node_limit=20000, bound_lp=blp, leaf_routing_warm=True).solve()
        assert res.routing_warm == getattr(lp, "routing_copies", 0)
        total += res.routing_warm
    assert total > 0


class _RefRootInfeasibleLP:
    """Wraps a StreamingOracleLP: the box with no fixings (the two-model search's reference root, REFROOT) is
    reported infeasible by presolve; every other box is solved as usual."""

    def __new__(cls, base):
        from oracle_lp import LP_INFEASIBLE
        orig = base.submit

        def submit(slots, lb=None, ub=None, **kw):
            st = orig(slots, lb, ub, **kw)
            for b, s in enumerate(np.asarray(slots).reshape(-1)):
                if lb is None or not np.isfinite(lb[b]).any():
                    base._pend.pop(int(s), None)
                    st[b] = LP_INFEASIBLE
            return st
        base.submit = submit
        return base


@pytest.mark.timeout(120)
def test_two_model_search_ends_when_refroot_is_presolve_infeasible():
    """a reference root (REFROOT) that presolve rejects used to leave the leaf engine 'not ready'
    forever, and with no time limit the loop spun with pending leaves and nothing in flight.  It must end:
    the leaves then start cold and the search still reaches the recorded MIP optimum (the other LPs here
    are solved normally)."""
    from core.engine.bnb import OPTIMAL, BranchAndBound
    from oracle_lp import StreamingOracleLP
    name, k = STEP1_N[0]
    p, data = _data(name)
    rec = G[name]["models"][k]
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    lp = _RefRootInfeasibleLP(StreamingOracleLP(data, variant, step=1, max_batch=10, alpha=alpha))
    blp = StreamingOracleLP(data, variant, step=1, max_batch=9, alpha=alpha, relaxation=1)
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                         batch=8, node_limit=20000, bound_lp=blp).solve()
    assert res.lp_status_kind["refroot"]["presolve_infeasible"] == 1
    if rec["status"] == 0:
        assert res.status == OPTIMAL, res.as_dict()
        assert _close(res.objective, rec["mip_objective"]), (res.objective, rec["mip_objective"])


def test_check_placement_budget_is_per_node():
    """C8 is n[j] * node_costs[j] <= node_budget per node (constraints_step1.py:101-103).  A
    placement opening more than budget / cost = 60 nodes (every source served locally at 70 nodes) meets
    every reference row and must pass the fp64 check (a summed budget rejected it)."""
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F = 70, 2
    data = data_to_solver_input(synthetic_payload(N, F, seed=0), with_db=False)
    step = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5)
    step.data = data
    C = np.ones((F, N))
    n = np.ones(N)
    x = np.zeros((F, N, N))
    x[:, np.arange(N), np.arange(N)] = 1.0
    assert float(np.asarray(data.node_costs) @ n) > data.node_budget      # the summed form would reject it
    assert step.check_placement(C, n, x)
    n_bad = n.copy()
    n_bad[0] = 0.0                                                          # C6 violated at node 0
    assert not step.check_placement(C, n_bad, x)
