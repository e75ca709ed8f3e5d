"""The whole NEPTUNE flow on the GPU at BASELINE config 2's, 3's and 4's sizes (VERDICT r4 item 6, r5 missing #3):
the reference's orchestration (core/solvers/neptune/neptune.py:18-39 — step 1, max_score = its objective, step-2
delete, and
create when delete does not end OPTIMAL) through the product's NeptuneMinDelayAndUtilization, every step's
branch-and-bound time-limited.  Checked on the host in fp64 against the reference's own rows:
  * step 1's placement meets every step-1 row (constraints_step1.py) and its score is the MDU objective of it
    (objectives.py:30-53);
  * the step-2 placement the flow returns meets every step-1 and step-2 row (constraints_step2.py) at the
    step-1 score, and its score is the disruption objective (objectives.py:55-63) of its integer vector;
  * the response the flow returns is the step-2 placement's wire format (output.py:23-39)."""
import numpy as np
import pytest

from scale_util import check_step1_solution, check_step2_solution

pytestmark = pytest.mark.gpu


def _dense_rows(x):
    """SparseRouting -> the aggregated routing rows [R, N] it stores (row_f, row_src)."""
    xb = np.zeros((len(x.row_f), x.N))
    xb[x.row, x.dst] = x.val
    return xb


def _flow(payload, seconds):
    import time
    from core.solvers.neptune.neptune import NeptuneMinDelayAndUtilization
    from core.utils import data_to_solver_input
    data = data_to_solver_input(payload, with_db=False)
    alpha = payload["solver"]["args"]["alpha"]
    t0 = time.time()
    solver = NeptuneMinDelayAndUtilization(alpha=alpha, time_limit=seconds, verbose=False)
    solver.load_data(data)
    solved = solver.solve()
    routing, alloc = solver.results()
    score = solver.score()
    s1, sd, sc = solver.step1.result, solver.step2_delete.result, solver.step2_create.result
    print(f"{len(data.nodes)}x{len(data.functions)}: {time.time() - t0:.1f} s; step 1 {s1.status} {s1.objective} "
          f"(bound {s1.bound}); delete {sd.status} {sd.objective}; create "
          f"{None if sc is None else (sc.status, sc.objective)}; score {score}")
    return data, alpha, solver, solved, alloc, score


def _check_step1(data, alpha, solver, score):
    """step 1: a feasible placement of the reference's step-1 rows whose MDU objective is the reported score"""
    s1 = solver.step1.result
    assert s1.objective is not None
    viol, worst, obj1 = check_step1_solution(data, "MinDelayAndUtilization", alpha, _dense_rows(s1.x), s1.x.row_f,
                                             s1.x.row_src, s1.z)
    assert worst <= 1e-6 and viol["C4"] <= 1e-6, viol
    assert abs(obj1 - score["step1"]) <= 1e-6 * max(1.0, abs(score["step1"])), (obj1, score)
    assert s1.bound <= score["step1"] + 1e-9


def _alloc_set(data, z, F, N):
    c = np.asarray(z[:F * N]).reshape(F, N) > 0.5
    return {(data.functions[k], data.nodes[j]) for k, j in zip(*np.nonzero(c))}


@pytest.mark.parametrize("n,f,seconds", [(64, 32, 20.0), (256, 128, 40.0), (512, 256, 45.0), (1024, 512, 45.0)])
def test_neptune_mdu_flow_end_to_end(n, f, seconds):
    """BASELINE config 5's shape (Alibaba trace: W == 0, D = 1 - I, 0.6 % of (f, j) pre-allocated) at config 2's,
    3's and its own size (1024 x 512, the whole neptune.py:18-39 orchestration on one GPU): step 2 is feasible (the published Alibaba flow: delete infeasible, create places every function
    on the fewest nodes keeping the most old placements), so every step of the flow is checked."""
    from core.utils.synthetic import alibaba_payload
    data, alpha, solver, solved, alloc, score = _flow(alibaba_payload(n, f, seed=0), seconds)
    _check_step1(data, alpha, solver, score)
    # step 2: the orchestration of neptune.py:24-39 — delete, then create unless delete ended OPTIMAL; the response
    # is the step-2 placement of the mode that solved, else step 1's; the score is delete's if it solved, else create's
    sd, sc = solver.step2_delete.result, solver.step2_create.result
    assert solver.step2_delete_solved == (sd.status == "OPTIMAL")
    assert (sc is None) == solver.step2_delete_solved
    took = sd if solver.step2_delete_solved else sc
    assert solved == (took.status == "OPTIMAL")
    got = {(fn, nd) for fn, d in alloc.items() for nd in d}
    assert got == _alloc_set(data, took.z if solved else solver.step1.result.z, f, n)
    found = [(mode, r) for mode, r in (("delete", sd), ("create", sc)) if r is not None and r.objective is not None]
    assert found, "no step-2 mode found a placement"
    for mode, r2 in found:
        # every placement a step-2 search returns is feasible for every step-1 and step-2 row at max_score = the
        # step-1 score, with its disruption objective (objectives.py:55-63) the reported one, above its bound
        viol, worst, obj2 = check_step2_solution(data, "MinDelayAndUtilization", alpha, mode, score["step1"],
                                                 _dense_rows(r2.x), r2.x.row_f, r2.x.row_src, r2.z)
        assert worst <= 1e-6 and viol["C4"] <= 1e-6, (mode, viol)
        assert abs(obj2 - r2.objective) <= 1e-6 * max(1.0, abs(r2.objective)), (mode, obj2, r2.objective)
        assert r2.bound <= r2.objective + 1e-9
        if r2 is took:
            assert abs(obj2 - score["step2"]) <= 1e-6 * max(1.0, abs(score["step2"])), (obj2, score)


@pytest.mark.parametrize("n,f,seconds", [(64, 32, 15.0), (256, 128, 30.0), (512, 256, 45.0)])
def test_neptune_mdu_flow_synthetic_generator(n, f, seconds):
    """The SURVEY §8(d) generator: its step-2 score row (constraints_step2.py:76-88, delays normalised by
    max(1000, max_k D[k, i]), not by step 1's MWD: SURVEY Appendix B #5) admits no placement within 1.3 x the
    step-1 score here, so both step-2 modes end without a placement and the flow returns step 1's placement with
    step 2's failed score, as the reference does (neptune.py:24-39)."""
    from core.utils.synthetic import synthetic_payload
    data, alpha, solver, solved, alloc, score = _flow(synthetic_payload(n, f, seed=0), seconds)
    _check_step1(data, alpha, solver, score)
    # both step-2 modes PROVEN infeasible (round-5 VERDICT: a time-limited LIMIT passed the same as a proof): the
    # reference falls back from delete to create and then returns step 1's placement (neptune.py:24-39)
    st = {m_: getattr(r, "status", None) for m_, r in (("delete", solver.step2_delete.result),
                                                        ("create", solver.step2_create.result))}
    print(f"{n}x{f} step 2:", st)
    assert st == {"delete": "INFEASIBLE", "create": "INFEASIBLE"}, st
    assert not solved and score["step2"] == 0.0
    got = {(fn, nd) for fn, d in alloc.items() for nd in d}
    assert got == _alloc_set(data, solver.step1.result.z, f, n)
