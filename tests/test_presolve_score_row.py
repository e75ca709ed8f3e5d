"""Node presolve of the step-2 score / delay row (csrc/nep_host.cpp score_row_xmin; DESIGN.md §4
"Infeasibility"): a node box whose closed placements push the row's smallest activity over the routing
simplexes above its right-hand side is infeasible.  Checked on every node box a branch-and-bound visits
on the reference's own step-2 models (the B&B runs on the oracle's HiGHS LPs, tests/oracle_lp.py):
each box HiGHS proves infeasible on the reference formulation is rejected by the presolve, no feasible
box is, and the from-scratch and incremental presolves agree.  Host code only (no GPU)."""
import numpy as np
import pytest

from golden_util import model, payload


@pytest.mark.parametrize("name,variant", [("syn_4x3_s0_r0.5_NeptuneMinDelay", "MinDelay"),
                                          ("syn_6x4_s1_r0.3_NeptuneMinDelay", "MinDelay")])
def test_score_row_presolve_matches_highs(name, variant):
    import core.engine.bnb as B
    from core.engine.lp import debug_presolve
    from core.utils import data_to_solver_input
    from oracle.solve import solve
    from oracle_lp import OracleLP
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    N, F = len(data.nodes), len(data.functions)
    nx = N * N * F
    m1 = model(name, 0)
    data.prev_x = m1["mip_x"][:nx].reshape(F, N, N).transpose(1, 0, 2)
    data.max_score = float(m1["mip_objective"])
    D, W = np.asarray(data.node_delay_matrix, float), np.asarray(data.workload_matrix, float)
    prev = float(np.sum(D[:, None, :] * W.T[:, :, None] * data.prev_x))
    lp = OracleLP(data, variant, step=2, max_batch=4, max_score=data.max_score)
    seen = []

    class Recording(B.BranchAndBound):
        def _submit(self, items, inc):
            seen.extend((node.idx.copy(), node.val.copy()) for _, _, node in items)
            return super()._submit(items, inc)

    Recording(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=2,
              node_limit=2000).solve()
    lb = np.full((len(seen), lp.n_int), -np.inf)
    ub = np.full((len(seen), lp.n_int), np.inf)
    for b, (idx, val) in enumerate(seen):
        lb[b, idx] = ub[b, idx] = val
    ok_full, ok_node, _, _ = debug_presolve(data, variant, lb, ub, step=2, max_score=data.max_score,
                                            prev_network_delay=prev)
    assert (ok_full == ok_node).all()
    infeasible = 0
    for b, (idx, val) in enumerate(seen):
        rl, ru = lp.m["lb"].copy(), lp.m["ub"].copy()
        rl[nx + idx] = val
        ru[nx + idx] = val
        st, _, _ = solve(lp.m, relax=True, lb=rl, ub=ru)
        if st == 2:
            infeasible += 1
            assert not ok_node[b], f"box {b}: HiGHS infeasible, presolve feasible"
        else:
            assert ok_node[b], f"box {b}: HiGHS feasible, presolve infeasible"
    assert infeasible > 0
