"""The native rounding heuristic (nep_round_leaf, csrc/nep_round.cpp; called by core/engine/bnb.py) gives the
same leaves, bit for bit, as the Python form it replaced (tests/round_ref.py): random node boxes (fixed-open
and fixed-closed c, n fixed either way), flows and LP c values — including ties, near-full memories and
nodes with no leaf — in all three rounding modes, with and without n."""
import types

import numpy as np
import pytest

from round_ref import RoundRef


def _case(rng, F, N, with_n):
    fn_mem = rng.integers(4, 33, size=F).astype(np.float64)
    node_mem = rng.integers(16, 96, size=N).astype(np.float64)
    flow = (rng.random((F, N)) * (rng.random((F, N)) < 0.3)).astype(np.float32)
    flow[rng.random((F, N)) < 0.05] = 0.5                       # ties
    zc = np.where(rng.random((F, N)) < 0.2, rng.choice([0.25, 0.5, 0.75, 1.0], size=(F, N)), 0.0)
    c0, c1 = 0, F * N
    n_range = (F * N, F * N + N) if with_n else None
    k = int(rng.integers(0, max(1, F * N // 4)))
    idx = rng.choice(F * N + (N if with_n else 0), size=k, replace=False)
    val = (rng.random(k) < 0.3).astype(np.float64)
    node = types.SimpleNamespace(idx=np.sort(idx).astype(np.int64), val=val[np.argsort(idx)])
    return RoundRef(F, N, c0, c1, n_range, fn_mem, node_mem), node, flow, zc


@pytest.mark.parametrize("with_n", [True, False])
def test_native_rounding_matches_reference(with_n):
    from core.engine.bnb import BranchAndBound
    rng = np.random.default_rng(7 if with_n else 8)
    seen = {"none": 0, "leaf": 0}
    for t in range(300):
        F, N = int(rng.integers(1, 9)), int(rng.integers(1, 13))
        ref, node, flow, zc = _case(rng, F, N, with_n)
        eng = BranchAndBound.__new__(BranchAndBound)
        eng.F, eng.N, eng.c0, eng.c1, eng.n_range = F, N, ref.c0, ref.c1, ref.n_range
        eng.fn_mem, eng.node_mem, eng.flow_tol = ref.fn_mem, ref.node_mem, ref.flow_tol
        eng.round_modes = ((False, None), (True, None), (True, 1.0 - 1e-6))
        for z in (zc.ravel(), None):   # the batched call (_round_all) gives the single-mode calls' leaves
            allm = eng._round_all(node, flow, z)
            for (by_flow, min_flow), b in zip(eng.round_modes, allm):
                a = eng._round(node, flow, z, by_flow, min_flow)
                assert (a is None and b is None) or (a is not None and b is not None and np.array_equal(a[0], b[0])
                                                     and np.array_equal(a[1], b[1]))
        for by_flow, min_flow in ((False, None), (True, None), (True, 1.0 - 1e-6)):
            for z in (zc.ravel(), None):
                a = ref._round(node, flow, z, by_flow, min_flow)
                b = eng._round(node, flow, z, by_flow, min_flow)
                if a is None:
                    assert b is None, (t, by_flow, min_flow)
                    seen["none"] += 1
                    continue
                assert b is not None, (t, by_flow, min_flow)
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (t, by_flow, min_flow)
                seen["leaf"] += 1
    assert seen["none"] > 0 and seen["leaf"] > 0, seen
