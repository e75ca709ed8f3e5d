"""The device-side helpers around a finished node LP (csrc/nep_aux.hip) against host computations on
the same engine solution:
  nep_lp_get_flows          flow[f, j] = sum_i x[i, f, j]  (the B&B's branching / rounding input)
  nep_lp_routing_entries    the wire format of neptune/utils/output.py:23-31 (x > 0.001, np.round(x, 3))
  nep_lp_allocation_entries output.py:33-39 (c > 0.001)
  nep_lp_score_check        efttc/utils/objectives.py scorers + constraints_step1.py checkers
"""
import numpy as np
import pytest

from gpu_cases import build_args

pytestmark = pytest.mark.gpu
CASES = [("payload", 0), ("syn_8x4_s2_r0.1_NeptuneMinDelayAndUtilization", 0), ("syn_10x5_s4_r0.2_NeptuneMinDelay", 0),
         ("sim5_NeptuneMinUtilization", 0)]


def _solved(name, k, fix_seed=3):
    from core.engine.lp import LPModel
    data, variant, step, kw = build_args(name, k)
    m = LPModel(data, variant, step=step, max_batch=3, **kw)
    F, N = len(data.functions), len(data.nodes)
    rng = np.random.default_rng(fix_seed)
    lb = np.full((3, m.n_int), -np.inf)
    ub = np.full((3, m.n_int), np.inf)
    for b in (1, 2):                           # a leaf-like node: every c fixed (a feasible rounding)
        c = np.zeros((F, N))
        for f in range(F):
            c[f, rng.integers(0, N)] = 1.0
        lb[b, :F * N] = ub[b, :F * N] = c.ravel()
    r = m.solve(np.arange(3), lb, ub, tol=1e-7, max_iters=50000)
    return m, data, variant, r


def _dense(m, data, slot):
    z, x = m.solution(slot, dense_x=True)
    return z, x.astype(np.float64)


@pytest.mark.parametrize("name,k", CASES)
def test_flows_entries_and_checks(name, k):
    m, data, variant, r = _solved(name, k)
    F, N = len(data.functions), len(data.nodes)
    try:
        for slot in range(3):
            if int(r["status"][slot]) == 2:
                continue
            z, x = _dense(m, data, slot)
            # flows
            fl = m.flows([slot])[0]
            ref = x.sum(axis=0)                             # [f, j]
            assert np.allclose(fl, ref, rtol=1e-6, atol=1e-6)
            # split flows (nep_lp_get_flows_split): the workload sources' part (W[f, i] > 0) of the same sum
            fl2, wfl = m.flows([slot], split=True)
            Wm = np.asarray(data.workload_matrix) > 0       # [f, i]
            wref = (x * Wm.T[:, :, None]).sum(axis=0)
            assert np.array_equal(fl2[0], fl)
            assert np.allclose(wfl[0], wref, rtol=1e-6, atol=1e-6)
            # routing entries == reference wire format of the dense x
            row, dst, val = m.routing_entries(slot)
            xb, rf, rs = m.rows(slot)
            W = np.asarray(data.workload_matrix)
            got = {}
            for rr, j, v in zip(row.tolist(), dst.tolist(), val.tolist()):
                srcs = [rs[rr]] if rs[rr] >= 0 else [i for i in range(N) if W[rf[rr], i] == 0]
                for i in srcs:
                    got[(i, int(rf[rr]), j)] = v
            ii, ff, jj = np.nonzero(x > 0.001)
            want = {(i, f, j): float(np.round(x[i, f, j], 3)) for i, f, j in zip(ii, ff, jj)}
            assert got == want
            # allocation entries
            fn, dj = m.allocation_entries(slot)
            cm = z[:F * N].reshape(F, N)
            assert sorted(zip(fn.tolist(), dj.tolist())) == sorted(zip(*np.nonzero(cm > 0.001)))
            # scorers / checkers
            sc = m.score_check(slot)
            D, cpr = np.asarray(data.node_delay_matrix), np.asarray(data.core_per_req_matrix)
            delay = float(np.sum(x * D[:, None, :] * W.T[:, :, None]))
            assert abs(sc["network_delay"] - delay) <= 1e-6 * max(1.0, abs(delay))
            flow = x.sum(axis=0)
            cb = cm != 0
            bad_cx = int(((flow > np.where(cb, 1e6, 0.0)) | (flow + 1e-6 < np.where(cb, 1.0, 0.0))).sum())
            assert sc["bad_c_x"] == bad_cx
            cpu = np.einsum("ifj,fi,fj->j", x, W, cpr)
            assert sc["bad_cpu"] == int((cpu > np.asarray(data.node_cores_matrix) + 1e-6).sum())
            mem = (np.asarray(data.function_memory_matrix)[:, None] * cb).sum(axis=0)
            assert sc["bad_memory"] == int((mem > np.asarray(data.node_memory_matrix)).sum())
            dev = np.abs(x.sum(axis=2) - 1.0)
            assert sc["bad_handle"] == int((~(dev < 0.1)).sum())
            if variant != "MinDelay":
                n = z[F * N:F * N + N]
                assert sc["nodes_used"] == int((n != 0).sum())
    finally:
        m.close()


@pytest.mark.parametrize("name,k", CASES[:2])
def test_batched_solutions_equal_single_reads(name, k):
    """nep_lp_get_solutions (API 8, the B&B's one read per advance) returns, slot for slot, what
    nep_lp_get_solution returns: the certified repaired point of a certified LP, else the iterate."""
    m, data, variant, r = _solved(name, k)
    try:
        zs = m.solutions([2, 0, 1])
        for row, slot in zip(zs, (2, 0, 1)):
            z, _ = m.solution(slot, dense_x=False)
            assert np.array_equal(row, z), slot
    finally:
        m.close()


@pytest.mark.parametrize("name,k", CASES[:2])
def test_copy_state_copies_every_slot_array(name, k):
    """nep_lp_copy_state copies a slot's iterate in one launch (nep_aux.hip copy_segments): afterwards the
    destination reads back exactly what the source does — repaired point, routing x, duals
    and the control block (status, iteration count, primal weight)."""
    from core.engine.lp import debug_build
    m, data, variant, r = _solved(name, k)
    try:
        _, _, step, kw = build_args(name, k)
        n_dual = debug_build(data, variant, step=step, **kw)["n_dual"]
        m.copy_state(0, 2)
        z0, x0 = m.solution(0)
        z2, x2 = m.solution(2)
        assert np.array_equal(z0, z2) and np.array_equal(x0, x2)
        assert np.array_equal(m.diag(0), m.diag(2))
        s0, s2 = m.debug_state(0, n_dual), m.debug_state(2, n_dual)
        assert np.array_equal(s0["y"], s2["y"])
    finally:
        m.close()
