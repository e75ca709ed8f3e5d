"""HiGHS parity on the node LPs an actual branch-and-bound visits (not random fixings): the product B&B
(core/engine/bnb.py) runs on the 64x32 synthetic instance (BASELINE config 2, step-1
MinDelayAndUtilization) for a few seconds, every node on the reference model (no bound_lp: the reference LP
at branching nodes too, the LP SCIP solves there); deep node boxes it finished are re-solved by HiGHS on the
reference formulation (oracle/):
  * certified LPs (NEP_LP_OPTIMAL; mostly rounding leaves, every c and n fixed) equal HiGHS within 1e-6;
  * bound-converged branching nodes (NEP_LP_BOUND) hold a valid bound (<= HiGHS + 1e-6) — printed with
    their gap;
  * LPs the engine proved infeasible (the Farkas test) are infeasible for HiGHS too."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_bnb_node_lps_match_highs():
    from core.engine import bnb as B
    from core.engine.lp import LP_BOUND, LP_INFEASIBLE, LP_OPTIMAL, LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve
    N, F = 64, 32
    p = synthetic_payload(N, F, seed=0)
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    rec = {LP_OPTIMAL: [], LP_BOUND: [], LP_INFEASIBLE: []}

    class Recording(B.BranchAndBound):
        def _finish(self, eng, slot, node, st, obj, pobj, iters, inc, *rest):
            if st in rec:
                rec[st].append((node.idx.copy(), node.val.copy(), obj))
            return super()._finish(eng, slot, node, st, obj, pobj, iters, inc, *rest)

    try:
        Recording(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=32, tol=5e-7,
                  time_limit=6.0, upper_bound=ub * (1 + 1e-6) + 1e-6, node_max_iters=1024, native=False).solve()
    finally:
        m.close()
    mdl = build_model(oracle_input(p, with_db=False), "MinDelayAndUtilization", step=1, alpha=0.5)
    nx = N * N * F

    def highs(idx, val):
        lb, ubb = mdl["lb"].copy(), mdl["ub"].copy()
        lb[nx + idx] = val
        ubb[nx + idx] = val
        st, obj, _ = solve(mdl, relax=True, lb=lb, ub=ubb)
        return st, obj

    def deepest(items, k):
        return sorted(items, key=lambda t: -len(t[0]))[:k]

    assert len(rec[LP_OPTIMAL]) > 0
    for idx, val, obj in deepest(rec[LP_OPTIMAL], 8):
        st, ref = highs(idx, val)
        assert st == 0, f"certified box ({len(idx)} fixings) is infeasible for HiGHS"
        assert abs(obj - ref) <= 1e-6 * max(1.0, abs(ref)), (len(idx), obj, ref)
    for idx, val, obj in deepest(rec[LP_BOUND], 6):
        st, ref = highs(idx, val)
        if st == 0:
            assert obj <= ref + 1e-6 * max(1.0, abs(ref)), (len(idx), obj, ref)
            print(f"bound-converged node ({len(idx)} fixings): bound {obj:.9g} HiGHS {ref:.9g} "
                  f"gap {(ref - obj) / max(1.0, abs(ref)):.2e}")
    for idx, val, _ in deepest(rec[LP_INFEASIBLE], 6):
        st, _ = highs(idx, val)
        assert st == 2, f"engine-infeasible box ({len(idx)} fixings) is feasible for HiGHS"
    print({k: len(v) for k, v in rec.items()})
