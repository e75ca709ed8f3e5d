"""The step-2 integral bound (core/solvers/neptune/neptune_step.py NeptuneStep2Base.integer_bound)
against brute force on the reference formulation: for every binary c that covers each function
(constraints_step1.py:5-35), minimize_disruption (objectives.py:55-63) is minimised over the integer
moved_from / moved_to / allocated / deallocated (variables.py:29-33, constraints_step2.py:5-54) by
enumeration.  The bound must never exceed the best completion of a node's fixings, must equal it on
complete fixings, and must be +inf exactly when no completion exists."""
import itertools
import math
import types

import numpy as np
import pytest


def _objective(c, old, mode):
    """min over the integer step-2 variables for a fixed binary c (None: infeasible)."""
    w = old.size
    A = int(((c == 1) & (old == 0)).sum())
    R = int(((c == 0) & (old == 1)).sum())
    O, C = int(old.sum()), int(c.sum())
    best = None
    for al in range(-w, 1):
        if al > O - C:
            continue
        for de in range(-w, 1):
            if de > C - O:
                continue
            if mode == "delete" and de + al + O - C < 0:
                continue
            if mode == "create" and de + al - O + C < 0:
                continue
            v = w * (A + R) + (w - 1) * al + (w + 1) * de
            best = v if best is None else min(best, v)
    return best


def _solver(F, N, old, mode):
    from core.solvers.neptune.neptune_step import NeptuneStep2Base
    s = NeptuneStep2Base.__new__(NeptuneStep2Base)
    s.mode = mode
    s.data = types.SimpleNamespace(functions=list(range(F)), nodes=list(range(N)),
                                   old_allocations_matrix=old.reshape(F, N).astype(float))
    return s.integer_bound()


@pytest.mark.parametrize("mode", ["delete", "create"])
@pytest.mark.parametrize("seed", range(6))
def test_step2_integer_bound_brute_force(mode, seed):
    rng = np.random.default_rng(seed)
    F, N = 2, 3
    FN = F * N
    old = (rng.random(FN) < 0.4).astype(int)
    bound = _solver(F, N, old, mode)
    values = {}
    for bits in itertools.product((0, 1), repeat=FN):
        c = np.array(bits)
        if (c.reshape(F, N).sum(axis=1) < 1).any():
            continue
        values[bits] = _objective(c, old, mode)
    # random partial fixings, plus the empty and every complete one
    fixings = [np.zeros(0, np.int64)] + [rng.permutation(FN)[:k] for k in range(1, FN) for _ in range(4)]
    for idx in fixings:
        for vals in itertools.product((0, 1), repeat=len(idx)):
            val = np.array(vals, float)
            comp = [v for bits, v in values.items() if v is not None
                    and all(bits[i] == int(x) for i, x in zip(idx, val))]
            b = bound(np.asarray(idx, np.int64), val)
            if not comp:
                continue                      # a bound may stay finite without a completion
            assert b <= min(comp) + 1e-9, (idx, val, b, min(comp))
    for bits, v in values.items():
        b = bound(np.arange(FN), np.array(bits, float))
        if v is None:
            assert b == math.inf, (bits, b)
        else:
            assert b == v, (bits, b, v)


@pytest.mark.parametrize("mode", ["delete", "create"])
@pytest.mark.parametrize("seed", range(4))
def test_step2_relocation_prices_exactly(mode, seed):
    """NeptuneStep2Base.improve: every neighbour it returns is a column exchange of the incumbent,
    fits memory, and its objective (the exact closed form, integer_bound on a complete fixing) is
    below the incumbent's; and it finds the best exchange (brute force over all pairs)."""
    from core.solvers.neptune.neptune_step import NeptuneStep2Base
    rng = np.random.default_rng(seed)
    F, N = 3, 5
    FN = F * N
    old = (rng.random((F, N)) < 0.35).astype(float)
    s = NeptuneStep2Base.__new__(NeptuneStep2Base)
    s.mode = mode
    s.data = types.SimpleNamespace(functions=list(range(F)), nodes=list(range(N)), old_allocations_matrix=old,
                                   function_memory_matrix=rng.integers(1, 4, F).astype(float),
                                   node_memory_matrix=rng.integers(3, 9, N).astype(float))
    bound = s.integer_bound()
    layout = {"c": (0, FN), "n": (FN + 4, FN + 4 + N)}
    imp = s.improve(layout, top=FN * N)
    for trial in range(20):
        P = (rng.random((F, N)) < 0.3).astype(float)
        P[np.arange(F), rng.integers(0, N, F)] = 1.0
        value = bound(np.arange(FN), P.ravel())
        if not np.isfinite(value) or (s.data.function_memory_matrix @ P > s.data.node_memory_matrix).any():
            continue                      # an incumbent is feasible
        idx = np.concatenate([np.arange(FN), np.arange(FN + 4, FN + 4 + N)])
        val = np.concatenate([P.ravel(), (P.sum(axis=0) > 0).astype(float)])
        got = imp(idx, val, value)
        mem = s.data.function_memory_matrix
        best = value
        for ju in range(N):
            for jt in range(N):
                if ju == jt or P[:, ju].sum() == 0:
                    continue
                Q = P.copy()
                Q[:, [ju, jt]] = Q[:, [jt, ju]]
                if (mem @ Q > s.data.node_memory_matrix + 1e-9).any():
                    continue
                best = min(best, bound(np.arange(FN), Q.ravel()))
        vals = []
        for gi, gv in got:
            Q = gv[:FN].reshape(F, N)
            assert sorted(map(tuple, Q.T.tolist())) == sorted(map(tuple, P.T.tolist()))   # an exchange
            assert (mem @ Q <= s.data.node_memory_matrix + 1e-9).all()
            assert np.array_equal(gv[FN:], (Q.sum(axis=0) > 0).astype(float))
            vals.append(bound(np.arange(FN), Q.ravel()))
            assert vals[-1] < value
        if best < value - 0.5:
            assert vals and min(vals) == best, (vals, best, value)
        else:
            assert not got


@pytest.mark.parametrize("mode", ["delete", "create"])
@pytest.mark.parametrize("seed", range(16))
def test_step2_integer_bound_with_node_cap(mode, seed):
    """MinUtilization step 2: at most K = max_score * soften nodes open (constraints_step2.py:71-73).
    Brute force over binary c (n = any c per node, n fixings respected): the bound never exceeds the
    best completion of a node's c / n fixings and is +inf when no completion exists."""
    from core.solvers.neptune.neptune_step import NeptuneStep2MinUtilization
    rng = np.random.default_rng(100 + seed)
    F, N = (2, 4) if seed < 8 else (3, 4)     # (round 5: the K-node cover bound on additions, kept old placements)
    FN = F * N
    old = (rng.random(FN) < 0.45).astype(int)
    s = NeptuneStep2MinUtilization.__new__(NeptuneStep2MinUtilization)
    s.mode, s.soften_step1_sol = mode, 1.0
    K = int(rng.integers(1, 3))
    s.data = types.SimpleNamespace(functions=list(range(F)), nodes=list(range(N)), max_score=K + 0.3,
                                   old_allocations_matrix=old.reshape(F, N).astype(float))
    n0 = 3 * FN + 2
    bound = s.integer_bound({"c": (0, FN), "n": (n0, n0 + N)})
    values = {}
    for bits in itertools.product((0, 1), repeat=FN):
        c = np.array(bits)
        opened = c.reshape(F, N).any(axis=0)
        if (c.reshape(F, N).sum(axis=1) < 1).any() or opened.sum() > K:
            continue
        values[bits] = (_objective(c, old, mode), opened)
    for _ in range(60):
        k = int(rng.integers(0, FN))
        ci = rng.permutation(FN)[:k]
        cv = rng.integers(0, 2, k).astype(float)
        kn = int(rng.integers(0, 3))
        ni = rng.permutation(N)[:kn]
        nv = rng.integers(0, 2, kn).astype(float)
        comp = [v for bits, (v, op) in values.items() if v is not None
                and all(bits[i] == int(x) for i, x in zip(ci, cv)) and all(op[j] == bool(x) for j, x in zip(ni, nv))]
        b = bound(np.concatenate([ci, n0 + ni]).astype(np.int64), np.concatenate([cv, nv]))
        if comp:
            assert b <= min(comp) + 1e-9, (ci, cv, ni, nv, b, min(comp))


@pytest.mark.parametrize("mode", ["delete", "create"])
@pytest.mark.parametrize("cap", [math.inf, 2.0, 3.0])
@pytest.mark.parametrize("seed", range(4))
def test_native_integer_bound_equals_python(mode, cap, seed):
    """The native tree's copy of integer_bound (csrc/nep_bnb.cpp step2_ibound, nep_bnb_debug_ibound) equals
    NeptuneStep2Base.integer_bound on random c / n boxes, with and without the node cap."""
    import ctypes
    from core.engine.lp import BnbParams, load_library
    from core.solvers.neptune.neptune_step import NeptuneStep2Base
    rng = np.random.default_rng(300 + seed)
    F, N = 4, 5
    FN = F * N
    old = (rng.random((F, N)) < 0.35).astype(float)
    s = NeptuneStep2Base.__new__(NeptuneStep2Base)
    s.mode = mode
    s.data = types.SimpleNamespace(functions=list(range(F)), nodes=list(range(N)), old_allocations_matrix=old)
    s.node_cap = lambda: cap
    n0 = FN + 3
    layout = {"c": (0, FN), "n": (n0, n0 + N)}
    bound = s.integer_bound(layout)
    lib = load_library()
    p = BnbParams(c0=0, c1=FN, n0=n0, n1=n0 + N, n_int=n0 + N, F=F, N=N)
    oldv = np.ascontiguousarray(old.ravel())
    out = ctypes.c_double()
    for trial in range(200):
        k = int(rng.integers(0, FN + N))
        pool = np.concatenate([np.arange(FN), np.arange(n0, n0 + N)])
        idx = np.sort(rng.choice(pool, size=k, replace=False)).astype(np.int32)
        val = rng.integers(0, 2, size=k).astype(np.float64)
        ref = bound(idx.astype(np.int64), val)
        assert lib.nep_bnb_debug_ibound(ctypes.byref(p), 1 if mode == "create" else 0, float(cap), oldv.ctypes.data,
                                        k, idx.ctypes.data, val.ctypes.data, ctypes.byref(out)) == 0
        assert out.value == ref or abs(out.value - ref) <= 1e-9 * max(1.0, abs(ref)), (idx, val, out.value, ref)
