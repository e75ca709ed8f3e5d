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
