"""The iteration blocks replay captured HIP graphs; tol and cutoff must still be the ones of the LPs'
own submit (DeviceView::prm in device memory), not the values current when a graph was captured."""
import math

import numpy as np
import pytest

from scale_util import case_model_args, gap, scale_cases

pytestmark = pytest.mark.gpu


def test_cutoff_and_tol_follow_each_submit():
    from core.engine.lp import LPModel, LP_CUTOFF, LP_OPTIMAL
    c = scale_cases()["syn128x64_MDU_s1"]
    ref = c["root"]["lp_objective"]
    data, variant, step, kw = case_model_args(c)
    m = LPModel(data, variant, step=step, max_batch=2, **kw)
    try:
        # 1. a cutoff below the LP value: the bound crosses it after many blocks (graphs captured)
        r = m.solve([0], tol=1e-7, cutoff=0.5 * ref, max_iters=400000, check_every=16)
        assert int(r["status"][0]) == LP_CUTOFF, r
        # 2. the same model, no cutoff: must certify (a replayed graph with the old cutoff would cut off)
        r = m.solve([1], tol=1e-7, cutoff=math.inf, max_iters=400000, check_every=16)
        assert int(r["status"][0]) == LP_OPTIMAL, r
        assert gap(float(r["obj"][0]), ref) <= 1e-6
        it_tight = int(r["iters"][0])
        # 3. a looser tolerance certifies no later than the tight one
        r = m.solve([0], tol=1e-4, cutoff=math.inf, max_iters=400000, check_every=16)
        assert int(r["status"][0]) == LP_OPTIMAL and int(r["iters"][0]) <= it_tight, (r, it_tight)
    finally:
        m.close()
