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
