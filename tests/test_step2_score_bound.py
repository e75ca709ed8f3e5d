"""The step-2 score-row integer bound (NeptuneStep2Base.score_row_lower_bound): it must never declare
a step-2 model infeasible that the reference's own recorded model (HiGHS MIP on the reference builders,
tests/golden) solves, and on the SURVEY §8(d) generator it proves both step-2 modes infeasible at the root (what
tests/test_gpu_flow.py's synthetic flow asserts on the GPU)."""
import numpy as np
import pytest

from golden_util import golden, payload

G = golden()
MDU = [n for n in G if isinstance(G[n], dict) and "models" in G[n] and n.endswith("NeptuneMinDelayAndUtilization")
       and G[n]["models"][0].get("status") == 0]


def _step2(data, mode, alpha, max_score, soften=1.3):
    from core.solvers.neptune.neptune_step import NeptuneStep2MinDelayAndUtilization
    s = NeptuneStep2MinDelayAndUtilization(mode=mode, alpha=alpha, soften_step1_sol=soften, verbose=False)
    data.max_score = max_score
    s.load_data(data)
    return s


@pytest.mark.parametrize("name", MDU)
def test_bound_never_cuts_a_recorded_feasible_step2(name):
    from core.utils import data_to_solver_input
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    args = p["solver"].get("args", {})
    ms = float(G[name]["models"][0]["mip_objective"])
    for k, m in enumerate(G[name]["models"][1:], start=1):
        mode = "delete" if m["mode"] == "step2_delete" else "create"
        s = _step2(data, mode, args.get("alpha", 0.5), ms, args.get("soften_step1_sol", 1.3))
        lb = s.score_row_lower_bound()
        rhs = ms * args.get("soften_step1_sol", 1.3)
        if m["status"] == 0:      # the recorded MIP has a placement: the bound must admit it
            assert lb <= rhs * (1 + 1e-9) + 1e-9, (name, mode, lb, rhs)
            assert s.node_cap() >= 0


@pytest.mark.parametrize("n,f,ms", [(64, 32, 0.13606), (256, 128, 0.16728)])
def test_bound_proves_synthetic_step2_infeasible(n, f, ms):
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    data = data_to_solver_input(synthetic_payload(n, f, seed=0), with_db=False)
    for mode in ("delete", "create"):
        s = _step2(data, mode, 0.5, ms)
        assert s.score_row_lower_bound() > 1.3 * ms
        assert s.node_cap() == -1.0
        # every box's integer bound is +inf: the root is never searched
        bound = s.integer_bound({"c": (0, f * n), "n": (3 * f * n + 2, 3 * f * n + 2 + n)})
        assert bound(np.zeros(0, np.int64), np.zeros(0)) == np.inf
