"""bench.py's replay stream (ReplayStream) on CPU with the oracle as node-LP backend (tests/oracle_lp.py): a
trace recorded from the product's two-model search (core/engine/bnb.py trace=, as tools/record_bnb_trace.py
records the 512x256 fixture) replayed (a) on the reference model — the headline stream — and (b) natively,
each box on the model the search ran it on.  Every recorded non-root LP completes exactly once per pass; a
leaf box gives the same LP value both ways (the same reference LP); a branching box's facility-relaxation
value is >= its reference-LP value (the relaxation is tighter); warm starts from a resident
parent state happen."""
import math
import types

import numpy as np
import pytest

from golden_util import golden, payload
from gpu_cases import VARIANT

G = golden()
CASES = [n for n in ("syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization", "syn_8x4_s3_r1.0_NeptuneMinUtilization")
         if n in G]


@pytest.mark.parametrize("name", CASES)
def test_replay_reference_and_native(name):
    import bench
    from core.engine.bnb import BranchAndBound
    from core.utils import data_to_solver_input
    from oracle_lp import LP_BOUND, LP_CUTOFF, LP_INFEASIBLE, LP_OPTIMAL, StreamingOracleLP
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    N, F = len(data.nodes), len(data.functions)
    trace = []
    lp = StreamingOracleLP(data, variant, step=1, max_batch=6, alpha=alpha)
    blp = StreamingOracleLP(data, variant, step=1, max_batch=5, alpha=alpha, relaxation=1)
    BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=4,
                   node_limit=20000, bound_lp=blp, trace=trace).solve()
    body = [e for e in trace if e["parent"] is not None]
    assert body and {e["model"] for e in trace} == {"leaf", "bound"}
    for e in trace:
        assert set(e) >= {"id", "kind", "model", "depth", "parent", "budget", "bound_res", "gap_tol", "cutoff"}
    a = types.SimpleNamespace(batch=4, tol=1e-6, max_iters=4096, check_every=12, warm_omega_floor=0.0,
                              functions=F, nodes=N)
    doc = {"lps": trace}
    runs = {}
    for native in (False, True):
        ref = StreamingOracleLP(data, variant, step=1, max_batch=5, alpha=alpha)
        fac = StreamingOracleLP(data, variant, step=1, max_batch=5, alpha=alpha, relaxation=1)
        for m in (ref, fac):
            m.solve([4])
        models = {"leaf": (ref, 4), "bound": (fac, 4)} if native else {"leaf": (ref, 4)}
        s = bench.ReplayStream(models, a, 0, 1, doc, native=native)
        s.drain(len(body))
        assert len(s.done) == len(body)
        assert s.counter == len(body)
        runs[native] = s
    if any(e["warm_from_parent"] and e["model"] == "leaf" for e in body):
        assert runs[False].warm_parent > 0
    # values per recorded entry: one slot per model, one node at a time (the streams above finish out of order)
    vals = {}
    for native in (False, True):
        ref = StreamingOracleLP(data, variant, step=1, max_batch=2, alpha=alpha)
        fac = StreamingOracleLP(data, variant, step=1, max_batch=2, alpha=alpha, relaxation=1)
        a1 = types.SimpleNamespace(**{**vars(a), "batch": 1})
        models = {"leaf": (ref, 1), "bound": (fac, 1)} if native else {"leaf": (ref, 1)}
        s = bench.ReplayStream(models, a1, 0, 1, doc, native=native)
        for k in range(len(body)):
            s.drain(1)
        vals[native] = s.done
    assert len(vals[False]) == len(vals[True]) == len(body)
    for e, r0, r1 in zip(body, vals[False], vals[True]):
        st0, o0 = r0[0], r0[1]
        st1, o1 = r1[0], r1[1]
        if st0 == LP_INFEASIBLE:
            assert st1 == LP_INFEASIBLE or e["model"] == "bound"
            continue
        if e["model"] == "leaf":
            assert st1 in (LP_OPTIMAL, LP_CUTOFF, LP_BOUND) and abs(o0 - o1) <= 1e-9 * max(1.0, abs(o0))
        elif st1 != LP_INFEASIBLE:
            assert o1 >= o0 - 1e-7 * max(1.0, abs(o0)), (e, o0, o1)
    assert math.isfinite(sum(r[1] for r in vals[False] if r[0] == LP_OPTIMAL))


@pytest.mark.parametrize("name", CASES)
def test_replay_parks_parent_states(name):
    """--park: a finished node whose children are still to come keeps its slot (its state parked) beyond the
    `batch` LPs in flight, so more nodes warm-start from their own parent; every LP still completes once, at
    most `batch` at a time, and the values are those of the unparked replay (the oracle solves each box from
    scratch, so only the slot bookkeeping differs)."""
    import bench
    from core.engine.bnb import BranchAndBound
    from core.utils import data_to_solver_input
    from oracle_lp import StreamingOracleLP
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    variant = VARIANT[p["solver"]["type"]]
    alpha = p["solver"].get("args", {}).get("alpha", 0.5)
    N, F = len(data.nodes), len(data.functions)
    trace = []
    lp = StreamingOracleLP(data, variant, step=1, max_batch=6, alpha=alpha)
    blp = StreamingOracleLP(data, variant, step=1, max_batch=5, alpha=alpha, relaxation=1)
    BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=4,
                   node_limit=20000, bound_lp=blp, trace=trace).solve()
    body = [e for e in trace if e["parent"] is not None]
    out = {}
    for park in (0, 8):
        a = types.SimpleNamespace(batch=2, tol=1e-6, max_iters=4096, check_every=12, warm_omega_floor=0.0,
                                  functions=F, nodes=N, park=park)
        ref = StreamingOracleLP(data, variant, step=1, max_batch=2 + park + 1, alpha=alpha)
        ref.solve([2 + park])
        s = bench.ReplayStream({"leaf": (ref, 2 + park)}, a, 0, 1, {"lps": trace})
        peak = [0]
        orig = ref.submit

        def submit(*args, **kw):
            r = orig(*args, **kw)
            peak[0] = max(peak[0], ref.active())
            return r
        ref.submit = submit
        s.drain(len(body))
        assert len(s.done) == len(body) and peak[0] <= 2
        assert len(s.depth) == len(s.done)
        out[park] = s
    assert out[8].warm_parent >= out[0].warm_parent
    assert sorted(r[1] for r in out[8].done) == sorted(r[1] for r in out[0].done)
