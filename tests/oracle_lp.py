"""Test-only stand-in for `core.engine.lp.LPModel` backed by the ORACLE: every node LP is HiGHS on
the reference's model restated as one CSR (oracle/formulation.py).  Lets the CPU suite run the
product's branch-and-bound (core/engine/bnb.py) and step orchestration (core/solvers) without a
GPU.  Routing rows are the literal per-(f, i) rows (no zero-workload pooling)."""
import math
import zlib

import numpy as np

from oracle.formulation import build_model
from oracle.solve import solve as oracle_solve

LP_OPTIMAL, LP_ITERATION_LIMIT, LP_INFEASIBLE, LP_CUTOFF, LP_BOUND = 0, 1, 2, 3, 5


class OracleLP:
    def __init__(self, data, variant, step=1, alpha=0.5, soften_step1_sol=1.3, max_score=0.0,
                 prev_network_delay=0.0, max_batch=1, relaxation=0):
        self.N, self.F = len(data.nodes), len(data.functions)
        self.variant = variant
        self.step = int(step)
        prev_x = getattr(data, "prev_x", None)
        if prev_x is None or not np.size(prev_x):
            prev_x = np.zeros((self.N, self.F, self.N))
        prev_x = np.asarray(prev_x, np.float64)
        self.m = build_model(data, variant, step=1 if self.step == 1 else 2,
                             mode="delete" if self.step == 2 else "create", alpha=alpha,
                             soften_step1_sol=soften_step1_sol, max_score=max_score, prev_x=prev_x)
        if relaxation:   # the B&B's facility relaxation (engine NEP_RELAX_FACILITY)
            from oracle.formulation import facility_relaxation
            self.m = facility_relaxation(self.m, data)
        self.nx = self.N * self.N * self.F
        self._W = np.asarray(data.workload_matrix, np.float64)
        self.n_int = self.m["A"].shape[1] - self.nx
        self.max_batch = max_batch
        self._sol = {}
        self.calls = 0

    def layout(self):
        FN, N = self.F * self.N, self.N
        has_n = self.variant != "MinDelay"
        if self.step == 1:
            return {"c": (0, FN), "n": (FN, FN + N) if has_n else None}
        out = {"c": (0, FN), "moved_from": (FN, 2 * FN), "moved_to": (2 * FN, 3 * FN),
               "allocated": (3 * FN, 3 * FN + 1), "deallocated": (3 * FN + 1, 3 * FN + 2)}
        out["n"] = (3 * FN + 2, 3 * FN + 2 + N) if has_n else None
        return out

    def solve(self, slots, lb=None, ub=None, tol=1e-7, cutoff=math.inf, max_iters=0, check_every=64,
              warm_start=False):
        slots = np.asarray(slots).reshape(-1)
        B = len(slots)
        obj = np.zeros(B)
        status = np.zeros(B, np.int32)
        for b, s in enumerate(slots):
            self.calls += 1
            rl, ru = self.m["lb"].copy(), self.m["ub"].copy()
            if lb is not None:
                fin = np.isfinite(lb[b])
                rl[self.nx:][fin] = np.maximum(rl[self.nx:][fin], lb[b][fin])
            if ub is not None:
                fin = np.isfinite(ub[b])
                ru[self.nx:][fin] = np.minimum(ru[self.nx:][fin], ub[b][fin])
            if (rl > ru).any():
                st, val, x = 2, None, None
            else:
                st, val, x = oracle_solve(self.m, relax=True, lb=rl, ub=ru)
            if val is None:
                status[b], obj[b] = LP_INFEASIBLE, math.inf
                self._sol[int(s)] = None
                continue
            obj[b] = val
            status[b] = LP_CUTOFF if val > cutoff else LP_OPTIMAL
            self._sol[int(s)] = x
        return {"obj": obj, "primal_obj": obj.copy(), "status": status, "iters": np.zeros(B, np.int64)}

    # streaming form (nep_lp_submit / nep_lp_advance): HiGHS solves each submitted node at once; advance
    # hands back up to min_done finished nodes per call, in slot order, like the engine's blocks
    def submit(self, slots, lb=None, ub=None, tol=1e-7, cutoff=math.inf, max_iters=0, check_every=64,
               warm_start=False, warm_omega_floor=0.0, bound_res=0.0, gap_tol=0.0, polish_after=0.0,
               warm_omega_cap=0.0):
        slots = np.asarray(slots).reshape(-1)
        self._cutoff = cutoff
        r = self.solve(slots, lb, ub, tol=tol, cutoff=math.inf)
        if not hasattr(self, "_queue"):
            self._queue = []
        st = np.zeros(len(slots), np.int32)
        for b, s in enumerate(slots):
            if int(r["status"][b]) == LP_INFEASIBLE:
                st[b] = LP_INFEASIBLE
                continue
            st[b] = LP_ITERATION_LIMIT
            self._queue.append((int(s), float(r["obj"][b])))
        return st

    def set_params(self, tol=1e-7, cutoff=math.inf):
        self._cutoff = cutoff

    def diag(self, slot):
        return {"pres": 0.0}

    def active(self):
        return len(getattr(self, "_queue", []))

    def advance(self, min_done=1):
        q = getattr(self, "_queue", [])
        k = len(q) if min_done <= 0 else min(len(q), max(1, int(min_done)))
        done, self._queue = sorted(q[:k]), q[k:]
        cut = getattr(self, "_cutoff", math.inf)
        obj = np.array([o for _, o in done])
        st = np.array([LP_CUTOFF if o > cut else LP_OPTIMAL for _, o in done], np.int32)
        return {"slots": np.array([s for s, _ in done], np.int32), "obj": obj, "primal_obj": obj.copy(),
                "status": st, "iters": np.zeros(len(done), np.int64)}

    def flows(self, slots, split=False):
        out = np.zeros((len(slots), self.F, self.N), np.float32)
        wout = np.zeros_like(out)
        for b, s in enumerate(np.asarray(slots).reshape(-1)):
            x = self._sol[int(s)][:self.nx].reshape(self.F, self.N, self.N)
            out[b] = x.sum(axis=1)
            wout[b] = (x * (self._W > 0)[:, :, None]).sum(axis=1)
        return (out, wout) if split else out

    def copy_state(self, src, dst):
        """Warm-start hand-off of the engine (nep_lp_copy_state); HiGHS solves from scratch, so this
        only records the copy (tests check the B&B's slot bookkeeping with it)."""
        self.copies = getattr(self, "copies", 0) + 1
        self._sol[int(dst)] = self._sol.get(int(src))

    def copy_routing_from(self, other, src, dst):
        """nep_lp_copy_routing: HiGHS has no routing state to take, so this records the hand-off only (the B&B
        tests check the two-model search issues it with a live bound-model slot)."""
        assert other is not self and other.N == self.N and other.F == self.F
        assert int(src) in other._sol, "routing warm start from a slot the bound model never solved"
        self.routing_copies = getattr(self, "routing_copies", 0) + 1

    def rows(self, slot):
        x = self._sol[int(slot)]
        xb = x[:self.nx].reshape(self.F * self.N, self.N).astype(np.float32)
        rf = np.repeat(np.arange(self.F), self.N).astype(np.int32)
        rs = np.tile(np.arange(self.N), self.F).astype(np.int32)
        return xb, rf, rs

    def solution(self, slot, dense_x=True):
        x = self._sol[int(slot)]
        z = x[self.nx:].copy()
        xd = x[:self.nx].reshape(self.F, self.N, self.N).transpose(1, 0, 2).astype(np.float32) if dense_x else None
        return z, xd

    def solutions(self, slots):
        return np.array([self.solution(s, dense_x=False)[0] for s in np.asarray(slots).reshape(-1)])

    def routing(self, slot):
        from core.engine.routing import SparseRouting
        return SparseRouting.from_dense(self.solution(slot, dense_x=True)[1])

    def row_map(self):
        """(row_f, row_src): one literal routing row per (f, i)"""
        return np.repeat(np.arange(self.F), self.N).astype(np.int32), np.tile(np.arange(self.N), self.F).astype(np.int32)

    def routing_from_entries(self, row, dst, val):
        from core.engine.routing import SparseRouting
        N, F = self.N, self.F
        return SparseRouting(N, F, np.repeat(np.arange(F), N), np.tile(np.arange(N), F), np.ones((F, N)), row, dst,
                             val)

    def close(self):
        self._sol = {}


class StreamingOracleLP(OracleLP):
    """OracleLP whose node LPs finish after a deterministic, node-dependent number of blocks (1-3
    advance() rounds, from a hash of the node box), so the branch-and-bound's streaming path sees LPs
    finish out of submission order as on the engine; and whose polish re-solve (tol <= 1e-8) reports
    a primal objective slightly ABOVE the certified one (the engine's polished value can land above
    the pre-polish incumbent: round-2 ADVICE)."""

    def submit(self, slots, lb=None, ub=None, tol=1e-7, cutoff=math.inf, max_iters=0, check_every=64,
               warm_start=False, warm_omega_floor=0.0, bound_res=0.0, gap_tol=0.0, polish_after=0.0,
               warm_omega_cap=0.0):
        slots = np.asarray(slots).reshape(-1)
        self._cutoff = cutoff
        r = self.solve(slots, lb, ub, tol=tol, cutoff=math.inf)
        if not hasattr(self, "_pend"):
            self._pend = {}
        st = np.zeros(len(slots), np.int32)
        for b, s in enumerate(slots):
            if int(r["status"][b]) == LP_INFEASIBLE:
                st[b] = LP_INFEASIBLE
                continue
            st[b] = LP_ITERATION_LIMIT
            key = np.concatenate([np.nan_to_num(lb[b], posinf=7, neginf=-7), np.nan_to_num(ub[b], posinf=7, neginf=-7)]) \
                if lb is not None else np.zeros(1)
            blocks = 1 + zlib.crc32(key.tobytes()) % 3   # deterministic across ranks
            obj = float(r["obj"][b])
            pobj = obj + (1e-9 * max(1.0, abs(obj)) if tol <= 1e-8 else 0.0)
            self._pend[int(s)] = [blocks, obj, pobj, bound_res > 0]   # bound_res: ends NEP_LP_BOUND
        return st

    def diag(self, slot):
        return {"pres": 0.0}

    def active(self):
        return len(getattr(self, "_pend", {}))

    def advance(self, min_done=1):
        pend = getattr(self, "_pend", {})
        done = []
        while pend:
            for s in sorted(pend):
                pend[s][0] -= 1
            fin = sorted(s for s in pend if pend[s][0] <= 0)
            done += [(s, pend.pop(s)) for s in fin]
            if min_done <= 0 or len(done) >= min_done:
                break
        cut = getattr(self, "_cutoff", math.inf)
        obj = np.array([v[1] for _, v in done])
        st = np.array([LP_CUTOFF if v[1] > cut else (LP_BOUND if v[3] else LP_OPTIMAL) for _, v in done], np.int32)
        return {"slots": np.array([s for s, _ in done], np.int32), "obj": obj,
                "primal_obj": np.array([v[2] for _, v in done]), "status": st,
                "iters": np.full(len(done), 12, np.int64)}
