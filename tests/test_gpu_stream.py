"""GPU: the streaming form of the engine (nep_lp_submit / nep_lp_advance — slots refilled as their
LP finishes, the way the B&B and bench.py keep every slot busy) certifies the same LP values as
HiGHS on the reference's recorded node LPs, with fewer slots than nodes."""
import numpy as np
import pytest

from gpu_cases import G, build_args, fixing_bounds

pytestmark = pytest.mark.gpu
TOL = 1e-6
CASES = [("payload", 0), ("syn_8x4_s2_r0.1_NeptuneMinDelayAndUtilization", 0), ("syn_6x4_s1_r0.3_NeptuneMinDelay", 0)]


@pytest.mark.parametrize("name,k", CASES)
def test_stream_refill_matches_highs(name, k):
    from core.engine.lp import LPModel, LP_INFEASIBLE, LP_OPTIMAL
    data, variant, step, kw = build_args(name, k)
    N, F = len(data.nodes), len(data.functions)
    m = LPModel(data, variant, step=step, max_batch=2, **kw)
    nodes = fixing_bounds(name, k, m.n_int, N * N * F)
    refs = [G[name]["models"][k]["lp_objective"]] + [r for _, _, r in nodes]
    queue = [(None, None)] + [(l[None], u[None]) for l, u, _ in nodes]
    got = {}
    where = {}
    nxt = 0

    def start(slot):
        nonlocal nxt
        while nxt < len(queue):
            b = nxt
            nxt += 1
            lb, ub = queue[b]
            st = m.submit([slot], lb, ub, tol=1e-7, max_iters=100000)
            if int(st[0]) == LP_INFEASIBLE:
                got[b] = (LP_INFEASIBLE, np.inf)
                continue
            where[slot] = b
            return

    for s in range(2):
        start(s)
    while m.active():
        r = m.advance(1)
        for i, s in enumerate(r["slots"]):
            got[where.pop(int(s))] = (int(r["status"][i]), float(r["obj"][i]))
            start(int(s))
    assert sorted(got) == list(range(len(queue)))
    for b, ref in enumerate(refs):
        st, obj = got[b]
        if ref is None:
            assert st != LP_OPTIMAL
            continue
        assert st == LP_OPTIMAL, (b, st, obj, ref)
        assert abs(obj - ref) <= TOL * max(1.0, abs(ref)), (b, obj, ref)
    m.close()


def test_submit_ex_per_lp_budgets_match_separate_submits():
    """API 12 nep_lp_submit_ex: the per-LP budgets of one call stop each LP where a submit of its own with that
    budget stops it (same status, iterations and values), and the unlimited ones certify the recorded LP value."""
    from core.engine.lp import LPModel, LP_ITERATION_LIMIT, LP_OPTIMAL
    name, k = "payload", 0
    data, variant, step, kw = build_args(name, k)
    ref = G[name]["models"][k]["lp_objective"]
    budgets = np.array([64, 100000, 128, 100000], np.int64)

    def run(per):
        m = LPModel(data, variant, step=step, max_batch=4, **kw)
        if per:
            st = m.submit(np.arange(4), None, None, tol=1e-7, max_iters=budgets, check_every=64,
                          bound_res=np.zeros(4))
        else:
            st = np.concatenate([m.submit([s], None, None, tol=1e-7, max_iters=int(budgets[s]), check_every=64)
                                 for s in range(4)])
        assert (st == LP_ITERATION_LIMIT).all()
        got = {}
        while m.active():
            r = m.advance(1)
            for i, s in enumerate(r["slots"]):
                got[int(s)] = (int(r["status"][i]), int(r["iters"][i]), float(r["obj"][i]),
                               float(r["primal_obj"][i]))
        m.close()
        return got

    per, sep = run(True), run(False)
    assert sorted(per) == [0, 1, 2, 3]
    for s in range(4):
        assert per[s][:2] == sep[s][:2], (s, per[s], sep[s])
        assert per[s][1] <= budgets[s]
        if per[s][0] == LP_ITERATION_LIMIT:
            assert per[s][1] == budgets[s]
    for s in (1, 3):
        assert per[s][0] == LP_OPTIMAL
        assert abs(per[s][2] - ref) <= TOL * max(1.0, abs(ref))



def test_copy_states_equals_copies_in_order():
    """API 12 nep_lp_copy_states: a chain of warm-start copies in one call (a destination read by a later pair, a
    source overwritten by a later pair) leaves every slot as the same copies made one nep_lp_copy_state at a time."""
    from core.engine.lp import LPModel
    name, k = "payload", 0
    data, variant, step, kw = build_args(name, k)
    src, dst = [0, 3, 1, 2, 4], [3, 4, 0, 5, 2]
    states = []
    for batched in (True, False):
        m = LPModel(data, variant, step=step, max_batch=6, **kw)
        lb = np.full((3, m.n_int), -np.inf)
        ub = np.full((3, m.n_int), np.inf)
        for b in range(3):
            lb[b, b] = ub[b, b] = 0.0
        m.solve(np.arange(3), lb, ub, tol=1e-7, max_iters=96, check_every=32)
        if batched:
            m.copy_states(src, dst)
        else:
            for a, b in zip(src, dst):
                m.copy_state(a, b)
        got = []
        for sl in range(6):
            z, _ = m.solution(sl, dense_x=False)
            d = m.diag(sl)
            got.append((sl, z.tobytes(), m.rows(sl)[0].tobytes(), d["omega"], d["k"]))
        if batched:   # (nep_lp_get_flows_solutions: the two reads of the tree's branching nodes in one round trip)
            fl, z = m.flows_solutions([5, 0, 2])
            assert np.array_equal(fl, m.flows([5, 0, 2])) and np.array_equal(z, m.solutions([5, 0, 2]))
        states.append(got)
        m.close()
    # the chain's expected sources: 0 <- 1, 2 <- 0 (via 3, 4), 3 <- 0, 4 <- 0, 5 <- 2
    assert states[0] == states[1]
    assert states[0][2][1:] == states[0][3][1:] == states[0][4][1:]
