"""core.engine.routing.SparseRouting — the routing solution as device-compacted entries of the engine's
aggregated rows — against the dense x[i][f][j] it stands for (reference `neptune/utils/output.py:5-39`):
the dense expansion, the wire format byte for byte (`convert_x_matrix` on the dense matrix), and the
step-2 MinDelay score-row constant (`constraints_step2.py:66-68`).  CPU only."""
import json

import numpy as np
import pytest

from core.engine.routing import SparseRouting
from core.solvers.neptune.output import convert_x_matrix


def _aggregated(seed, N=7, F=4):
    """A random aggregated-row solution: per f one row per loaded source + one pooled row (W == 0)."""
    rng = np.random.default_rng(seed)
    W = rng.integers(0, 3, size=(F, N)).astype(float) * (rng.random((F, N)) < 0.5)
    W[0] = 0.0                                         # a function with only the pooled row
    rf, rs, rows = [], [], []
    for f in range(F):
        for i in range(N):
            if W[f, i] != 0:
                rf.append(f)
                rs.append(i)
        if (W[f] == 0).any():
            rf.append(f)
            rs.append(-1)
    R = len(rf)
    xb = np.zeros((R, N), np.float32)
    for r in range(R):
        k = int(rng.integers(1, 4))
        j = rng.choice(N, size=k, replace=False)
        v = rng.random(k).astype(np.float32)
        v[0] = 0.0005 if r % 5 == 0 else v[0]          # an entry under the wire threshold
        xb[r, j] = v / v.sum()
    # dense reference
    dense = np.zeros((N, F, N))
    for r in range(R):
        srcs = [rs[r]] if rs[r] >= 0 else np.flatnonzero(W[rf[r]] == 0).tolist()
        for i in srcs:
            dense[i, rf[r]] = xb[r].astype(np.float64)
    row, dst = np.nonzero(xb)
    return SparseRouting(N, F, rf, rs, W, row, dst, xb[row, dst].astype(np.float64)), dense, W


@pytest.mark.parametrize("seed", range(4))
def test_dense_expansion_and_wire_format(seed):
    sr, dense, _ = _aggregated(seed)
    assert sr.shape == dense.shape and sr.size == dense.size
    np.testing.assert_array_equal(np.asarray(sr), dense)
    nodes = [f"n{i}" for i in range(dense.shape[0])]
    fns = [f"ns/f{f}" for f in range(dense.shape[1])]
    a = convert_x_matrix(sr, nodes, fns)
    b = convert_x_matrix(dense, nodes, fns)
    assert json.dumps(a) == json.dumps(b)             # same keys, values and insertion order


@pytest.mark.parametrize("seed", range(4))
def test_network_delay_matches_dense(seed):
    sr, dense, W = _aggregated(seed)
    N = dense.shape[0]
    D = np.random.default_rng(seed + 9).integers(0, 50, size=(N, N)).astype(float)
    ref = float(np.einsum("ij,fi,ifj->", D, W, dense))
    assert abs(sr.network_delay(D, W) - ref) <= 1e-12 * max(1.0, abs(ref))


def test_from_dense_round_trip_and_empty():
    _, dense, _ = _aggregated(11)
    np.testing.assert_array_equal(np.asarray(SparseRouting.from_dense(dense)), dense)
    e = SparseRouting.empty(3, 2)
    assert np.asarray(e).shape == (3, 2, 3) and not np.asarray(e).any()
    assert convert_x_matrix(e, ["a", "b", "c"], ["x/1", "x/2"]) == {}


def _overloaded(seed, N=8, F=4):
    """A leaf routing whose CPU rows exceed the cores by a certificate-sized relative amount (~1e-5)."""
    rng = np.random.default_rng(seed)
    W = rng.integers(1, 6, size=(F, N)).astype(float)
    W[np.arange(F), rng.integers(0, N, F)] = 0.0         # one zero-workload source per f: a pooled row
    cpr = rng.uniform(0.01, 0.1, size=(F, N))
    c_open = rng.random((F, N)) < 0.3
    c_open[:, 0] = True                                  # every function has >= 2 open destinations
    c_open[:, 1] = True
    c_open[:, 2] = True                                  # a destination every function may use, with room
    rf, rs = [], []
    for f in range(F):
        for i in range(N):
            if W[f, i] != 0:
                rf.append(f)
                rs.append(i)
        if (W[f] == 0).any():
            rf.append(f)
            rs.append(-1)
    rf, rs = np.array(rf), np.array(rs)
    xb = np.zeros((len(rf), N))
    for r in range(len(rf)):
        js = np.flatnonzero(c_open[rf[r]])
        v = rng.random(js.size) + 0.1
        xb[r, js] = v / v.sum()
    row, dst = np.nonzero(xb)
    x = SparseRouting(N, F, rf, rs, W, row, dst, xb[row, dst])
    if (np.asarray(x).sum(axis=0)[c_open] < 1.05).any():   # an LP leaf meets C2: open columns carry >= 1
        return _overloaded(seed + 1000, N, F)
    cpu = x.cpu_usage(W, cpr)
    cores = cpu * (1 + 1e-6 * rng.uniform(0, 1, N) - 0.5e-6)     # about half the nodes overloaded
    cores[2] = 2.0 * cpu.max()                                     # room there
    return x, W, cpr, cores, c_open


@pytest.mark.parametrize("seed", range(6))
def test_repair_cpu_meets_absolute_checker(seed):
    """core.engine.routing.repair_cpu: every node's CPU ends <= cores (the reference checker
    efttc/utils/constraints_step1.py:68-78 allows + 1e-6), every source row still sums to 1 (C4), flow
    only moves to open destinations (C1), open columns keep >= 1 (C2), and the returned cost change is
    sum coef * dx."""
    from core.engine.routing import repair_cpu
    x, W, cpr, cores, c_open = _overloaded(seed)
    N, F = x.N, x.F
    D = np.random.default_rng(seed + 3).integers(1, 40, size=(N, N)).astype(float)
    coef = lambda f, i, j: W[f, i] * D[i, j]
    assert (x.cpu_usage(W, cpr) > cores).any()
    x2, delta, ok = repair_cpu(x, W, cpr, cores, c_open, coef=coef)
    assert ok
    d0, d1 = np.asarray(x), np.asarray(x2)
    assert np.all(np.einsum("ifj,fi,fj->j", d1, W, cpr) <= cores)
    np.testing.assert_allclose(d1.sum(axis=2), d0.sum(axis=2), atol=1e-12)
    assert not (d1.transpose(1, 0, 2)[~c_open[:, None, :].repeat(N, 1)] > 0).any()
    col0, col1 = d0.sum(axis=0), d1.sum(axis=0)            # [f, j]
    assert np.all(col1[c_open] >= np.minimum(col0[c_open], 1.0) - 1e-12)
    ref = float(np.einsum("ifj,fi,ij->", d1 - d0, W, D))
    assert abs(delta - ref) <= 1e-12 * max(1.0, abs(ref))
    assert np.abs(d1 - d0).max() < 1e-4                   # certificate-sized moves only


def test_repair_cpu_noop_and_infeasible():
    from core.engine.routing import repair_cpu
    x, W, cpr, cores, c_open = _overloaded(0)
    big = np.full_like(cores, 1e9)
    x2, delta, ok = repair_cpu(x, W, cpr, big, c_open)
    assert x2 is x and delta == 0.0 and ok
    tiny = x.cpu_usage(W, cpr) * (1 - 1e-3)                  # every node overloaded: nowhere to move
    _, _, ok = repair_cpu(x, W, cpr, tiny, c_open)
    assert not ok


@pytest.mark.parametrize("seed", range(4))
def test_repair_cpu_keeps_step2_score_row(seed):
    """Step 2 (round-3 ADVICE): with the score / delay row's coefficients as `coef` and its room
    rhs + 1e-6 - activity (constraints_step2.py:57-88; the checker's tolerance,
    efttc/utils/constraints_step2.py:68, :95), the moves never raise the row beyond that room; with no
    room left only moves that lower it are taken, and ok = False when none is admissible."""
    from core.engine.routing import repair_cpu
    x, W, cpr, cores, c_open = _overloaded(seed)
    N = x.N
    D = np.random.default_rng(seed + 7).integers(1, 40, size=(N, N)).astype(float)
    coef = lambda f, i, j: W[f, i] * D[i, j]
    d0 = np.asarray(x)
    x_free, delta_free, ok_free = repair_cpu(x, W, cpr, cores, c_open, coef=coef)
    assert ok_free
    room = 0.5 * max(delta_free, 0.0)
    x2, delta, ok = repair_cpu(x, W, cpr, cores, c_open, coef=coef, score_room=room)
    d1 = np.asarray(x2)
    ref = float(np.einsum("ifj,fi,ij->", d1 - d0, W, D))
    assert abs(delta - ref) <= 1e-12 * max(1.0, abs(ref))
    assert delta <= room + 1e-12                                 # the row's room is respected
    if ok:
        assert np.all(np.einsum("ifj,fi,fj->j", d1, W, cpr) <= cores)
    _, delta0, _ = repair_cpu(x, W, cpr, cores, c_open, coef=coef, score_room=0.0)
    assert delta0 <= 1e-12                                        # no room: only non-increasing moves
