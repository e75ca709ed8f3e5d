"""CPU checks of the at-scale parity machinery: the host solution checker used on full-size GPU
solutions (scale_util.check_step1_solution) reproduces HiGHS's objective on a HiGHS solution with no
violations, and flags a corrupted one; tests/golden/scale.json is well-formed and its 64x32 root value
re-derives from the oracle."""
import numpy as np
import pytest

from scale_util import check_step1_solution, gap, scale_cases


def _highs_rows(N, F, seed, variant):
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve
    p = synthetic_payload(N, F, seed=seed, rho=0.3)
    data = data_to_solver_input(p, with_db=False)
    m = build_model(oracle_input(p, with_db=False), variant, step=1, alpha=0.5)
    st, obj, z = solve(m, relax=True)
    assert st == 0
    W = data.workload_matrix
    x = z[:N * N * F].reshape(F, N, N)              # [f, i, j]
    rows, rf, rs = [], [], []
    for f in range(F):
        zs = []
        for i in range(N):
            if W[f, i] != 0:
                rows.append(x[f, i]); rf.append(f); rs.append(i)
            else:
                zs.append(x[f, i])
        if zs:                                       # pooled zero-workload row: their mean (exact aggregation)
            rows.append(np.mean(zs, axis=0)); rf.append(f); rs.append(-1)
    return data, np.array(rows), np.array(rf), np.array(rs), z[N * N * F:], obj


@pytest.mark.parametrize("variant", ["MinDelayAndUtilization", "MinDelay", "MinUtilization"])
def test_checker_on_highs_solution(variant):
    data, xb, rf, rs, z, obj = _highs_rows(12, 5, 3, variant)
    viol, worst, hobj = check_step1_solution(data, variant, 0.5, xb, rf, rs, z)
    assert viol["C4"] <= 1e-8 and worst <= 1e-7, viol
    assert abs(hobj - obj) <= 1e-9 * max(1.0, abs(obj)), (hobj, obj)
    bad = xb.copy()
    bad[0] *= 1.01                                   # breaks C4 for that row
    assert check_step1_solution(data, variant, 0.5, bad, rf, rs, z)[0]["C4"] > 1e-3


def test_scale_fixture_well_formed():
    cs = scale_cases()
    for k in ("syn64x32_MDU_s1", "syn128x64_MDU_s1", "syn256x128_MDU_s1", "alibaba_MinDelayAndUtilization_s1",
              "alibaba_MinUtilization_s2create"):
        assert k in cs, k
    for name, c in cs.items():
        assert c["root"]["status"] == 0 and c["root"]["lp_objective"] is not None, name
        for nd in c["nodes"]:
            assert len(nd["fix_idx"]) == len(nd["fix_val"]) and all(0 <= i < c["n_int"] for i in nd["fix_idx"])
            assert (nd["lp_objective"] is None) == (nd["status"] != 0)


def test_scale_fixture_64x32_root_rederives():
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import solve
    from scale_util import case_payload
    c = scale_cases()["syn64x32_MDU_s1"]
    p = case_payload(c)
    m = build_model(oracle_input(p, with_db=False), "MinDelayAndUtilization", step=1, alpha=0.5)
    nx = 64 * 64 * 32
    nd = c["nodes"][3]
    lb, ub = m["lb"].copy(), m["ub"].copy()
    lb[nx + np.array(nd["fix_idx"])] = nd["fix_val"]
    ub[nx + np.array(nd["fix_idx"])] = nd["fix_val"]
    st, obj, _ = solve(m, relax=True, lb=lb, ub=ub)
    assert st == 0 and gap(obj, nd["lp_objective"]) <= 1e-9
