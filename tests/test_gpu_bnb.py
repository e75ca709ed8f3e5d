"""The product's streaming branch-and-bound (core/engine/bnb.py) on the MI355X engine at BASELINE
config 2/3/4 sizes (64x32, 256x128, 512x256 on one GPU), time-limited: it must return a feasible placement whose objective it reports
correctly, a valid bound, and device-side helpers (flows, scorer/checker) consistent with it.  And
the NeptuneWithEFTTC* flows (EF-TTC step 1 + the NEPTUNE step-2 MIP on the GPU) reproduce the
reference's recorded scores (tests/golden/efttc.json)."""
import json
import math
import os

import numpy as np
import pytest

from golden_util import GOLDEN

pytestmark = pytest.mark.gpu


def _mdu_objective(data, alpha, x, z):
    """objectives.py:30-53 on a placement (dense x[i,f,j], z = c[F*N] + n[N])."""
    W, D = np.asarray(data.workload_matrix, float), np.asarray(data.node_delay_matrix, float)
    md = np.asarray(data.max_delay_matrix, float)
    F, N = W.shape
    obj = alpha / N * float(np.sum(z[F * N:F * N + N]))
    if W.sum():
        mwd = 0.0
        for mdv in np.unique(md):
            best = np.where(D <= mdv, D, -np.inf).max(axis=1)
            mwd += float((W[md == mdv] * best[None, :]).sum())
        obj += (1 - alpha) / mwd * float(np.sum(x * D[:, None, :] * W.T[:, :, None]))
    return obj


@pytest.mark.parametrize("n,f,seconds", [(64, 32, 25.0), (256, 128, 40.0), (512, 256, 90.0)])
def test_product_bnb_time_limited(n, f, seconds):
    from core.engine.bnb import INFEASIBLE, BranchAndBound
    from core.engine.lp import LPModel
    from core.solvers.efttc import scoring
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    p = synthetic_payload(n, f, seed=0)
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    bm = None
    try:
        if n < 512:   # the one-model search (every node LP on the reference model)
            res = BranchAndBound(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                                 batch=32, tol=5e-7, time_limit=seconds, root_max_iters=200000,
                                 upper_bound=ub * (1 + 1e-6) + 1e-6, repair=st1.routing_repair(m.layout())).solve()
        else:         # the product's step-1 search at config 4 (facility-relaxation bounds, the capacity-greedy
            # root heuristic; NeptuneStepBase.branch_and_bound): the one-model search's rounding
            # leaves can all fail the presolve's CPU cover here, depending on which optimal face the root lands on
            st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6,
                                                        lp_max_iters=4096)
            st1.load_data(data)
            bm = st1.bound_model(data, 33)
            res = st1.branch_and_bound(m, bm, time_limit=seconds, root_max_iters=400000).solve()
    finally:
        m.close()
        if bm is not None:
            bm.close()
    print(res.as_dict())
    # a stop decision ends the search within a block of the LPs in flight (they stop at their next check)
    assert res.seconds <= seconds + 30.0, res.as_dict()
    assert res.status != INFEASIBLE and res.objective is not None, res.as_dict()
    assert res.certified > 0 and res.nodes > 0
    assert res.bound <= res.objective + 1e-9
    if n >= 512:
        # config 4's product search (facility-relaxation bounds): a proven gap, not only an incumbent (round-5
        # VERDICT; the bench's 60 s figure is 2.5 %)
        rel = (res.objective - res.bound) / max(1.0, abs(res.objective))
        assert rel <= 0.05, (rel, res.as_dict())
    x, z = np.asarray(res.x, np.float64), np.asarray(res.z, np.float64)
    c = z[:f * n].reshape(f, n)
    assert np.all((np.abs(c) < 1e-9) | (np.abs(c - 1) < 1e-9)), "incumbent c not integral"
    # the incumbent's objective, recomputed on the host, is the reported one
    assert abs(_mdu_objective(data, 0.5, x, z) - res.objective) <= 1e-6 * max(1.0, abs(res.objective))
    # and it is feasible by the reference's own checker at its ABSOLUTE tolerance (efttc/utils/
    # constraints_step1.py:68-78: CPU <= cores + 1e-6), polished or not: the returned routing went through
    # the CPU repair (core.engine.routing.repair_cpu)
    assert res.repaired, res.as_dict()
    assert scoring.cpu_usage_ok(data, x)
    mem = (np.asarray(data.function_memory_matrix)[:, None] * (c > 0.5)).sum(axis=0)
    assert np.all(mem <= np.asarray(data.node_memory_matrix) + 1e-9)
    assert np.all(np.abs(x.sum(axis=2) - 1.0) <= 1e-6)       # C4 at the parity bar


with open(os.path.join(GOLDEN, "efttc.json")) as fh:
    E = json.load(fh)
WITH = sorted(k for k in E if k.split("|")[1].startswith("NeptuneWithEFTTC") and "error" not in E[k]
              and k.split("|")[0] in ("payload", "testpy", "sim0_NeptuneMinDelay", "sim3_NeptuneMinUtilization",
                                      "syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization"))


@pytest.mark.parametrize("key", WITH)
def test_neptune_with_efttc_flow_on_gpu(key):
    import core.solvers as S
    from core.utils import data_to_solver_input
    name, stype = key.split("|")
    with open(os.path.join(GOLDEN, "inputs", name + ".json")) as fh:
        p = json.load(fh)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    solver = S.SOLVERS[stype](**p["solver"].get("args", {}))
    solver.load_data(data)
    solver.solve()
    score = solver.score()
    ref = E[key]["response"]["score"]
    assert math.isclose(score["step1"], ref["step1"], rel_tol=1e-9, abs_tol=1e-9), (score, ref)
    assert abs(score["step2"] - ref["step2"]) <= 1e-6 * max(1.0, abs(ref["step2"])), (score, ref)


PUBLISHED = {"NeptuneMinDelay": {"step1": 0.0, "step2": 23.0},
             "NeptuneMinDelayAndUtilization": {"step1": 0.005, "step2": 65010.0},
             "NeptuneMinUtilization": {"step1": 1.0, "step2": 65010.0}}


@pytest.mark.parametrize("stype", sorted(PUBLISHED))
def test_alibaba_flow_matches_recorded_scip_scores(stype):
    """The reference's Alibaba 100x25 trace case (testing/alibaba/alibaba_test/output_<solver>_case0.json:
    scores recorded with SCIP in 436 / 1258 / 1225 s) through the product solver on the GPU, each step's
    B&B limited to 30 s: both step scores must equal the recorded ones (tied optima: scores only)."""
    import time
    import core.solvers as S
    from core.utils import data_to_solver_input
    with open(os.path.join(GOLDEN, "inputs", f"alibaba_{stype}.json")) as fh:
        p = json.load(fh)
    args = dict(p["solver"].get("args", {}))
    args.update(time_limit=30.0, verbose=False)
    t0 = time.time()
    solver = S.SOLVERS[stype](**args)
    solver.load_data(data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False))
    solver.solve()
    score = solver.score()
    print(stype, score, f"{time.time() - t0:.1f} s")
    for k, ref in PUBLISHED[stype].items():
        assert abs(score[k] - ref) <= 1e-6 * max(1.0, abs(ref)), (stype, score, PUBLISHED[stype])
