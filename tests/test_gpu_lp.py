"""GPU parity: the MI355X LP engine's certified LP values equal HiGHS on the reference's own
recorded models (root LPs of every step model, and seeded B&B-node fixings), within 1e-6."""
import numpy as np
import pytest

from gpu_cases import G, build_args, fixing_bounds, lp_cases

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _gap(a, b):
    return abs(a - b) / max(1.0, abs(b))


@pytest.mark.parametrize("name,k", lp_cases())
def test_root_and_node_lps(name, k):
    from core.engine.lp import LPModel, LP_OPTIMAL, LP_INFEASIBLE
    data, variant, step, kw = build_args(name, k)
    rec = G[name]["models"][k]
    nodes = G[name]['models'][k].get('node_lps', [])
    m = LPModel(data, variant, step=step, max_batch=1 + len(nodes), **kw)
    N, F = len(data.nodes), len(data.functions)
    nx = N * N * F
    nodes = fixing_bounds(name, k, m.n_int, nx)
    B = 1 + len(nodes)
    lb = np.full((B, m.n_int), -np.inf)
    ub = np.full((B, m.n_int), np.inf)
    for b, (l, u, _) in enumerate(nodes):
        lb[b + 1], ub[b + 1] = l, u
    res = m.solve(np.arange(B), lb, ub, max_iters=100000)
    refs = [rec["lp_objective"]] + [r for _, _, r in nodes]
    for b, ref in enumerate(refs):
        st, obj = int(res["status"][b]), float(res["obj"][b])
        if ref is None:
            assert st != LP_OPTIMAL, f"node {b}: HiGHS infeasible but engine says optimal obj={obj}"
            continue
        assert st == LP_OPTIMAL, f"node {b}: status {st} iters {res['iters'][b]} obj {obj} ref {ref}"
        assert _gap(obj, ref) <= TOL, f"node {b}: obj {obj} ref {ref} primal {res['primal_obj'][b]}"
