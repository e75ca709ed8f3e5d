"""The native tree search (csrc/nep_bnb.cpp, API 12) on CPU: the engine library's tree drives HiGHS node LPs
(tests/oracle_lp.py) through a Python call table (core/engine/lp.PyBnbEngine -> nep_bnb_create_engines), so the
C++ search — heap, queues, prune / branch / round, warm-start sources, the sharded search's frontier deal, per-loop
collective and rebalance — is exercised without a GPU.  The Python loop (core/engine/bnb.py, native=False) is the
reference: both must reach the recorded MIP optimum of the reference's own models, visit the same tree on one rank,
and deal the same frontier (crc32) when sharded over gloo, world 2."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from golden_util import golden, payload
from gpu_cases import VARIANT

G = golden()
STEP1 = [n for n in ("syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization", "syn_8x4_s2_r0.1_NeptuneMinDelay",
                     "sim5_NeptuneMinUtilization", "syn_8x4_s3_r1.0_NeptuneMinUtilization") if n in G]


def _setup(name, streaming=True, max_batch=6):
    from core.utils import data_to_solver_input
    from oracle_lp import OracleLP, StreamingOracleLP
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    args = p["solver"].get("args", {})
    cls = StreamingOracleLP if streaming else OracleLP
    lp = cls(data, VARIANT[p["solver"]["type"]], step=1, max_batch=max_batch, alpha=args.get("alpha", 0.5))
    return data, lp


def _search(name, native, comm=None, **kw):
    from core.engine.bnb import BranchAndBound
    data, lp = _setup(name)
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=4,
                         node_limit=20000, native=native, comm=comm, **kw).solve()
    return res


@pytest.mark.parametrize("name", STEP1)
def test_native_tree_on_highs_matches_python_loop(name):
    rec = G[name]["models"][0]
    py = _search(name, False)
    nat = _search(name, True)
    assert nat.native and not py.native
    assert nat.status == py.status == ("OPTIMAL" if rec["status"] == 0 else "INFEASIBLE")
    if rec["status"] == 0:
        assert abs(nat.objective - rec["mip_objective"]) <= 1e-6 * max(1.0, abs(rec["mip_objective"]))
        assert nat.objective == py.objective
        assert np.array_equal(nat.z, py.z)
    # the same decisions in the same order: the same tree
    assert (nat.nodes, nat.leaves, nat.lps) == (py.nodes, py.leaves, py.lps)
    assert nat.lp_status == py.lp_status


def test_native_tree_create_rejects_bad_parameters():
    import ctypes
    from core.engine.lp import BnbParams, PyBnbEngine, load_library
    lib = load_library()
    data, lp = _setup(STEP1[0])
    e = PyBnbEngine(lp, lp.F, lp.N)
    L = lp.layout()
    fm = np.ones(lp.F)
    nm = np.ones(lp.N)
    p = BnbParams(c0=L["c"][0], c1=L["c"][1], n0=-1, n1=-1, n_int=lp.n_int, F=lp.F, N=lp.N, batch=0, batch_b=1,
                  world=1, rank=0, tol=1e-6)
    assert not lib.nep_bnb_create_engines(ctypes.byref(e.table), None, ctypes.byref(p), fm.ctypes.data,
                                          nm.ctypes.data)
    assert b"batch" in lib.nep_last_error()
    p.batch, p.world, p.rank = 2, 2, 2
    assert not lib.nep_bnb_create_engines(ctypes.byref(e.table), None, ctypes.byref(p), fm.ctypes.data,
                                          nm.ctypes.data)
    assert b"rank" in lib.nep_last_error()


@pytest.mark.timeout(120)
def test_native_tree_ends_when_no_slot_can_free():
    """Round-5 ADVICE: warm starts off with one working slot — after the first LP incumbent keeps that slot no
    open node can ever be submitted; the search must end (LIMIT, the incumbent kept), not loop forever."""
    from core.engine.bnb import BranchAndBound
    name = "sim5_NeptuneMinUtilization"
    data, lp = _setup(name, max_batch=3)
    res = BranchAndBound(lp, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, batch=4,
                         node_limit=20000, native=True, warm=False).solve()
    assert res.status in ("LIMIT", "OPTIMAL")
    assert res.objective is not None


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, name, native, rebalance_every, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(os.path.dirname(here), "neptune-mip_amd"), os.path.dirname(here)]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from core.engine.comm import TorchComm
    res = _search(name, native, comm=TorchComm(), rebalance_every=rebalance_every, time_limit=600.0)
    x = None if res.x is None else np.asarray(res.x).round(12).tolist()
    out[(native, rank)] = (res.status, res.objective, None if res.z is None else np.asarray(res.z).tolist(), x,
                           res.split_hash, res.rebalanced, res.native)
    dist.destroy_process_group()


def _sharded(name, native, rebalance_every=8):
    with mp.Manager() as mgr:
        out = mgr.dict()
        mp.spawn(_worker, args=(2, _port(), name, native, rebalance_every, out), nprocs=2, join=True)
        return dict(out)


@pytest.mark.parametrize("name", STEP1[:3])
def test_sharded_native_tree_matches_recorded_mip(name):
    rec = G[name]["models"][0]
    nat = _sharded(name, True)
    st0, obj0, z0, x0, h0, _, native = nat[(True, 0)]
    assert native
    for r in range(2):
        assert nat[(True, r)][:4] == (st0, obj0, z0, x0), (r, nat[(True, r)][:2])
        assert nat[(True, r)][4] == h0, "the ranks dealt different frontiers"
    if rec["status"] == 0:
        assert st0 == "OPTIMAL"
        assert abs(obj0 - rec["mip_objective"]) <= 1e-6 * max(1.0, abs(rec["mip_objective"]))
    else:
        assert st0 == "INFEASIBLE"
    # before the split both loops run the same batch-synchronous search: the same frontier, the same crc32
    py = _sharded(name, False)
    assert py[(False, 0)][4] == h0


def test_sharded_native_tree_rebalances_idle_ranks():
    name = "sim5_NeptuneMinUtilization"
    rec = G[name]["models"][0]
    nat = _sharded(name, True, rebalance_every=1)
    for r in range(2):
        assert nat[(True, r)][:4] == nat[(True, 0)][:4]
    assert nat[(True, 0)][0] == "OPTIMAL"
    assert abs(nat[(True, 0)][1] - rec["mip_objective"]) <= 1e-6 * max(1.0, abs(rec["mip_objective"]))
    print("nodes received by rebalancing per rank:", [nat[(True, r)][5] for r in range(2)])
    assert sum(nat[(True, r)][5] for r in range(2)) > 0, "no rank ever took nodes from another"


@pytest.mark.parametrize("branching", [0, 2])
def test_native_tree_per_lp_budgets_merge_submit_groups(monkeypatch, branching):
    """API 12 submit_ex / copy_states: with per-LP budgets / bound stops the tree submits once per (engine, warm,
    check_every) group instead of once per (budget, bound stop) too — strong-branching probes, children and re-solves
    go in one call — and makes a submit's warm-start copies in one call.  The search must end where the per-budget,
    per-copy form ends (same status, objective and vector)."""
    import core.engine.lp as lpmod
    made = []

    class Rec(lpmod.PyBnbEngine):
        def __init__(self, model, F, N, per_lp=True):
            super().__init__(model, F, N, per_lp=per_lp)
            made.append(self)

    name = "syn_8x4_s3_r1.0_NeptuneMinUtilization" if "syn_8x4_s3_r1.0_NeptuneMinUtilization" in G else STEP1[0]
    out = {}
    for per_lp in (True, False):
        made.clear()
        Rec.__init__.__defaults__ = (per_lp,)
        monkeypatch.setattr(lpmod, "PyBnbEngine", Rec)
        res = _search(name, True, branching=branching)
        out[per_lp] = (res.status, res.objective, None if res.z is None else np.asarray(res.z).tolist())
        assert made and (made[0].ex_calls > 0) == per_lp
        assert (made[0].copies_calls > 0) == per_lp   # (warm-start copies through copy_states)
    assert out[True] == out[False]
