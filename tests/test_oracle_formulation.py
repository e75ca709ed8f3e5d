"""The oracle's restated CSR equals, entry by entry, the model the reference's own builders
recorded (tests/golden/models, tools/gen_golden.py)."""
import numpy as np
import pytest

from golden_util import golden, model, model_names, payload
from oracle.formulation import build_model
from oracle.inputs import data_to_solver_input

G = golden()
VARIANT = {"NeptuneMinDelayAndUtilization": "MinDelayAndUtilization", "NeptuneMinDelay": "MinDelay",
           "NeptuneMinUtilization": "MinUtilization"}


def _rebuild(name, k):
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    variant = VARIANT[p["solver"]["type"]]
    args = p["solver"].get("args", {})
    alpha = args.get("alpha", 0.5)
    soften = args.get("soften_step1_sol", 1.3)
    if k == 0:
        return build_model(data, variant, step=1, alpha=alpha)
    m1 = model(name, 0)
    F, N = data.workload_matrix.shape
    max_score = float(m1["mip_objective"])
    prev_x = m1["mip_x"][:N * N * F].reshape(F, N, N).transpose(1, 0, 2)   # -> [i,f,j]
    mode = "delete" if k == 1 else "create"
    return build_model(data, variant, step=2, mode=mode, alpha=alpha, soften_step1_sol=soften,
                       max_score=max_score, prev_x=prev_x)


def canonical(m):
    """Rows are recorded up to sign (the recorder's `a >= b` may arrive as `b <= a` when b is a
    Variable subclass); flip every row whose first nonzero is negative."""
    A = m["A"].tocsr().copy()
    A.sort_indices()
    lo, hi = m["lo"].copy(), m["hi"].copy()
    first = np.array([A.data[A.indptr[r]] if A.indptr[r + 1] > A.indptr[r] else 1.0 for r in range(A.shape[0])])
    flip = first < 0
    import scipy.sparse as sp
    S = sp.diags(np.where(flip, -1.0, 1.0))
    lo2 = np.where(flip, -hi, lo)
    hi2 = np.where(flip, -lo, hi)
    return dict(m, A=(S @ A).tocsr(), lo=lo2, hi=hi2)


@pytest.mark.parametrize("name,k", model_names())
def test_restated_model_equals_recorded(name, k):
    ref = canonical(model(name, k))
    got = canonical(_rebuild(name, k))
    assert got["A"].shape == ref["A"].shape
    diff = abs(got["A"] - ref["A"]).max() if got["A"].nnz else 0.0
    assert diff <= 1e-12 * max(1.0, abs(ref["A"]).max())
    for key in ("lo", "hi", "lb", "ub"):
        a, b = got[key], ref[key]
        assert np.array_equal(np.isinf(a), np.isinf(b)), key
        fin = np.isfinite(a)
        np.testing.assert_allclose(a[fin], b[fin], rtol=1e-12, atol=1e-15, err_msg=key)
    assert got["lo"].shape == ref["lo"].shape
    np.testing.assert_allclose(got["c"], ref["c"], rtol=1e-12, atol=0)
    assert np.array_equal(got["integrality"], ref["integrality"])
