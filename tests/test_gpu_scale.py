"""GPU parity at the BASELINE.json sizes.

1. tests/golden/scale.json (HiGHS on the reference formulation, tools/gen_scale_golden.py): the root LP
   and seeded B&B-node LPs of
     * the §8(d) synthetic generator at 64x32 (config 2), 128x64 and 256x128 (config 3);
     * the reference's Alibaba 100x25 trace case (W == 0: the R = F aggregation path), all three variants,
       and its step-2 create model at the published step-1 scores;
   solved as the B&B does: root first, then every node warm-started from the root's state.  Every LP
   must certify (NEP_LP_OPTIMAL) with |obj - HiGHS| <= 1e-6 * max(1, |HiGHS|); a node HiGHS proves
   infeasible must not be reported optimal.
2. Full-size root LPs no CPU reference can solve here (512x256: 67 M columns; the Alibaba-shape
   1024x512): certified, and the engine's solution re-checked on the host in fp64 against every
   reference row family (scale_util.check_step1_solution), its objective recomputed from x and z.
"""
import numpy as np
import pytest

from scale_util import case_model_args, check_step1_solution, gap, node_bounds, scale_cases

pytestmark = pytest.mark.gpu
TOL = 1e-6
SOLVE_TOL = 5e-7      # certificate tolerance of the solves: below the 1e-6 parity bar
C4_TOL = 1e-6         # fp32 routing rows: |sum_j x - 1| of the stored state, at the parity bar (logged: <= 3e-7)
CASES = scale_cases()


def _solve_case(c, tol=SOLVE_TOL):
    from core.engine.lp import LPModel
    data, variant, step, kw = case_model_args(c)
    B = len(c["nodes"])
    m = LPModel(data, variant, step=step, max_batch=B + 1, **kw)
    root = B
    rr = m.solve([root], tol=tol, max_iters=400000)
    lb, ub = node_bounds(c, m.n_int)
    for b in range(B):
        m.copy_state(root, b)
    res = m.solve(np.arange(B), lb, ub, tol=tol, max_iters=200000, warm_start=True)
    return m, rr, res


def _check_lp(what, st, obj, iters, ref):
    """Certified (NEP_LP_OPTIMAL) and within 1e-6 of HiGHS.  (Round 4 listed two 64x32 step-2 models whose LPs
    did not certify, KNOWN_UNCERTIFIED; the reduced disruption block certifies them)"""
    from core.engine.lp import LP_OPTIMAL
    assert st == LP_OPTIMAL, f"{what}: status {st} after {iters} iterations (HiGHS {ref})"
    assert gap(obj, ref) <= TOL, f"{what}: {obj} vs HiGHS {ref}"


@pytest.mark.parametrize("name", sorted(CASES))
def test_scale_parity(name):
    from core.engine.lp import LP_OPTIMAL
    c = dict(CASES[name], name=name)
    m, rr, res = _solve_case(c)
    try:
        _check_lp("root", int(rr["status"][0]), float(rr["obj"][0]), rr["iters"][0], c["root"]["lp_objective"])
        for b, nd in enumerate(c["nodes"]):
            st, obj = int(res["status"][b]), float(res["obj"][b])
            if nd["lp_objective"] is None:
                assert st != LP_OPTIMAL, f"node {b}: HiGHS infeasible, engine optimal {obj}"
                continue
            _check_lp(f"node {b}", st, obj, res["iters"][b], nd["lp_objective"])
        print(f"{name}: root {rr['iters'][0]} iterations, nodes {res['iters'].tolist()}")
    finally:
        m.close()


def _full_size_check(payload, variant, fixings=0, seed=0, boxes_fn=None, min_child_iters=0):
    """Root + `fixings` warm children (2 random c-fixings each, or the boxes boxes_fn(F, N, n_int) returns), every
    LP certified and re-checked on the host; children must run more than min_child_iters iterations."""
    from core.engine.lp import LPModel, LP_OPTIMAL
    from core.utils import data_to_solver_input
    data = data_to_solver_input(payload, with_db=False)
    alpha = payload["solver"]["args"]["alpha"]
    F, N = data.workload_matrix.shape
    custom = None
    if boxes_fn is not None:
        custom = boxes_fn(F, N)
        fixings = len(custom)
    B = 1 + fixings
    m = LPModel(data, variant, step=1, alpha=alpha, max_batch=B)
    try:
        rr = m.solve([0], tol=TOL, max_iters=400000)      # the bench's certificate tolerance
        assert int(rr["status"][0]) == LP_OPTIMAL, f"root: status {rr['status'][0]} after {rr['iters'][0]}"
        boxes = [(None, None)]
        if fixings:
            rng = np.random.default_rng(seed)
            lb = np.full((fixings, m.n_int), -np.inf)
            ub = np.full((fixings, m.n_int), np.inf)
            for b in range(fixings):
                if custom is not None:
                    idx, val = custom[b]
                    lb[b, idx] = ub[b, idx] = val
                else:
                    idx = rng.choice(F * N, size=2, replace=False)
                    lb[b, idx] = ub[b, idx] = rng.integers(0, 2, size=2)
                m.copy_state(0, b + 1)
            r2 = m.solve(np.arange(1, B), lb, ub, tol=TOL, max_iters=20000, warm_start=True)
            boxes += [(lb[b], ub[b]) for b in range(fixings)]
        for b in range(B):
            st = int(rr["status"][0]) if b == 0 else int(r2["status"][b - 1])
            its = int(rr["iters"][0]) if b == 0 else int(r2["iters"][b - 1])
            assert st == LP_OPTIMAL, f"LP {b}: status {st} after {its} iterations (every full-size LP must certify)"
            if b:
                assert its > min_child_iters, f"child {b}: certified after {its} iterations (its fixings force no work)"
            obj = float(rr["obj"][0]) if b == 0 else float(r2["obj"][b - 1])
            pobj = float(rr["primal_obj"][0]) if b == 0 else float(r2["primal_obj"][b - 1])
            xb, rf, rs = m.rows(b)
            z, _ = m.solution(b, dense_x=False)
            viol, worst, hobj = check_step1_solution(data, variant, alpha, xb, rf, rs, z, *boxes[b])
            print(f"LP {b}: {its} iterations, host fp64 re-check: worst row violation {worst:.2e} (C4 {viol['C4']:.2e})",
                  {k: f"{v:.1e}" for k, v in viol.items()})
            assert obj <= pobj + 1e-12, (obj, pobj)
            assert pobj - obj <= TOL * max(1.0, abs(obj)), (obj, pobj)
            # C4 (sum_j x = 1) is the fp32 routing state itself: the projection's fp32 threshold leaves each
            # row sum within a few fp32 ulps of the row's values (C4_TOL); every other row family at 1e-6
            assert viol["C4"] <= C4_TOL, viol
            assert worst <= TOL, viol
            assert abs(hobj - pobj) <= 1e-6 * max(1.0, abs(pobj)), (hobj, pobj)
        return rr
    finally:
        m.close()


def test_full_size_512x256_root_and_children():
    """BASELINE config 4's instance (512x256, §8(d) generator, seed 0): root + 4 warm children."""
    from core.utils.synthetic import synthetic_payload
    rr = _full_size_check(synthetic_payload(512, 256, seed=0), "MinDelayAndUtilization", fixings=4)
    print("512x256 root iterations", rr["iters"][0], "obj", rr["obj"][0])


def _alibaba_children(variant):
    """Children of the Alibaba-shape root that force the routing to move (the root certifies at iteration 1: with
    W == 0 every routing is free and its value only depends on n >= sum_f c / M, so a box that only closes
    destinations is certified at its first check — the round-5 children).  C2 (constraints_step1.py:5-15:
    sum_i x[i,f,j] >= c[f,j] - eps) makes a placement fixed open need a unit of flow, i.e. the pooled
    zero-workload row of f (weight N) must send >= 1/N of its mass there: every destination of 4 functions fixed
    open (their pooled rows exactly uniform); 4 functions open on the first half of the nodes with the second
    half closed (uniform on that half); every function restricted to two destinations, both open (each >= 1/N);
    10 nodes forced open and 8 functions open everywhere.  MinDelay has no n: the same c boxes."""
    has_n = variant != "MinDelay"

    def boxes(F, N):
        n0 = F * N
        out = []
        allj = np.arange(N)
        out.append(((np.arange(4)[:, None] * N + allj[None, :]).ravel(), np.ones(4 * N)))
        half = N // 2
        idx = [(np.arange(10, 14)[:, None] * N + allj[None, :half]).ravel()]
        val = [np.ones(4 * half)]
        if has_n:
            idx.append(n0 + np.arange(half, N))
            val.append(np.zeros(N - half))
        else:
            idx.append((np.arange(10, 14)[:, None] * N + allj[None, half:]).ravel())
            val.append(np.zeros(4 * (N - half)))
        out.append((np.concatenate(idx), np.concatenate(val)))
        keep = np.stack([np.arange(F) % N, (np.arange(F) + 1) % N], axis=1)
        closed = np.ones((F, N), bool)
        closed[np.arange(F), keep[:, 0]] = closed[np.arange(F), keep[:, 1]] = False
        opened = np.concatenate([np.arange(F) * N + keep[:, 0], np.arange(F) * N + keep[:, 1]])
        out.append((np.concatenate([np.flatnonzero(closed.ravel()), opened]),
                    np.concatenate([np.zeros(int(closed.sum())), np.ones(2 * F)])))
        idx = [(np.arange(20, 28)[:, None] * N + allj[None, :]).ravel()]
        val = [np.ones(8 * N)]
        if has_n:
            idx.append(n0 + np.arange(10))
            val.append(np.ones(10))
        out.append((np.concatenate(idx), np.concatenate(val)))
        return out
    return boxes


@pytest.mark.parametrize("variant", ["MinDelayAndUtilization", "MinUtilization", "MinDelay"])
def test_full_size_alibaba_1024x512(variant):
    """BASELINE config 5's shape (Alibaba trace: W == 0, D = 1 - I, R = F aggregated rows): root + children with
    the fixings of _alibaba_children.  The step-1 LP of this shape is degenerate: with W == 0 the objective is
    alpha / N sum n with n >= sum_f c / M, so every routing the projection onto a box's allowed destinations
    produces is optimal within 1e-6 once its repaired point is feasible — root and children certify at their first
    check (measured: 1 iteration each, cold or warm, even with every destination of a function forced open).  The
    check is the certificate itself and the host fp64 re-check of every reference row at 1024 x 512; the LPs that
    must iterate at this shape are step 2's (test_full_size_alibaba_1024x512_step2_create, 65-257 iterations)
    and the whole flow (tests/test_gpu_flow.py, 1024 x 512)."""
    from core.utils.synthetic import alibaba_payload
    rr = _full_size_check(alibaba_payload(1024, 512, seed=0), variant, boxes_fn=_alibaba_children(variant))
    print("1024x512", variant, "root iterations", rr["iters"][0], "obj", rr["obj"][0])


def test_full_size_alibaba_1024x512_step2_create():
    """BASELINE config 5's shape, step 2 (create, MinDelayAndUtilization at the published step-1 score
    0.005, gen_scale_golden.py:33): the root (optimum ~0: every function keeps its old placements) and 4
    warm children whose fixings force moves, so their optimum is O(1) .. O(F N): open 2 new (f, j) (cost
    1 each), close an old one (2 F N - 1 plus the opening it forces), empty a node (n = 0), move one
    function.  Each LP certified after more than one iteration and re-checked on the host in fp64 against
    every step-1 and step-2 row family, its disruption objective recomputed from z
    (scale_util.check_step2_solution; constraints_step2.py, objectives.py:55-63)."""
    from core.engine.lp import LPModel, LP_OPTIMAL, STEP2_CREATE
    from core.utils import data_to_solver_input
    from core.utils.synthetic import alibaba_payload
    from scale_util import check_step2_solution
    data = data_to_solver_input(alibaba_payload(1024, 512, seed=0), with_db=False)
    F, N = data.workload_matrix.shape
    FN = F * N
    old = np.asarray(data.old_allocations_matrix, np.float64)
    m = LPModel(data, "MinDelayAndUtilization", step=STEP2_CREATE, alpha=0.5, max_score=0.005,
                soften_step1_sol=1.3, max_batch=5)
    try:
        rr = m.solve([0], tol=TOL, max_iters=400000)
        assert int(rr["status"][0]) == LP_OPTIMAL, f"root: status {rr['status'][0]} after {rr['iters'][0]}"
        rng = np.random.default_rng(3)
        fs = [f for f in rng.permutation(F) if 0 < old[f].sum() < N][:4]
        ones = [np.flatnonzero(old[f] == 1) for f in fs]
        zeros = [np.flatnonzero(old[f] == 0) for f in fs]
        n0 = 3 * FN + 2
        j_node = int(np.flatnonzero(old.sum(axis=0) > 0)[0])
        fix = [([fs[0] * N + zeros[0][0], fs[0] * N + zeros[0][1]], [1.0, 1.0]),     # open two new placements
               ([fs[1] * N + ones[1][0]], [0.0]),                                     # close an old one
               ([n0 + j_node], [0.0]),                                                # empty a node
               ([fs[3] * N + ones[3][0], fs[3] * N + zeros[3][0]], [0.0, 1.0])]       # move a function
        lb = np.full((4, m.n_int), -np.inf)
        ub = np.full((4, m.n_int), np.inf)
        for b, (idx, val) in enumerate(fix):
            lb[b, idx] = ub[b, idx] = val
            m.copy_state(0, b + 1)
        r2 = m.solve(np.arange(1, 5), lb, ub, tol=TOL, max_iters=200000, warm_start=True)
        print("1024x512 step-2 create: root", rr["iters"][0], "its obj", rr["obj"][0], "; children its",
              r2["iters"].tolist(), "obj", r2["obj"].tolist())
        boxes = [(None, None)] + [(lb[b], ub[b]) for b in range(4)]
        for b in range(5):
            st = int(rr["status"][0]) if b == 0 else int(r2["status"][b - 1])
            obj = float(rr["obj"][0]) if b == 0 else float(r2["obj"][b - 1])
            pobj = float(rr["primal_obj"][0]) if b == 0 else float(r2["primal_obj"][b - 1])
            its = int(rr["iters"][0]) if b == 0 else int(r2["iters"][b - 1])
            assert st == LP_OPTIMAL, f"LP {b}: status {st} after {its} iterations"
            assert pobj - obj <= TOL * max(1.0, abs(obj)), (b, obj, pobj)
            if b:
                assert its > 1 and obj >= 0.5, f"child {b}: {its} iterations, objective {obj} (expected a forced move)"
            xb, rf, rs = m.rows(b)
            z, _ = m.solution(b, dense_x=False)
            viol, worst, hobj = check_step2_solution(data, "MinDelayAndUtilization", 0.5, "create", 0.005, xb, rf, rs,
                                                     z, *boxes[b])
            print(f"LP {b}: host fp64 re-check: worst {worst:.2e} (C4 {viol['C4']:.2e})")
            assert viol["C4"] <= C4_TOL and worst <= TOL, (b, viol)
            assert abs(hobj - pobj) <= 1e-6 * max(1.0, abs(pobj)), (b, hobj, pobj)
    finally:
        m.close()
