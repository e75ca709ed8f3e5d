"""Batched best-first branch-and-bound over the MI355X LP engine.

This is the tree search SCIP runs inside `pywraplp.Solver.Solve()` (reference
`core/solvers/solver.py:35-40`) on the NEPTUNE step models, rebuilt around batched GPU LP
relaxations: open nodes, heuristic completions and leaves are all LPs solved by `LPModel.solve`
(nep_lp_solve_batch), up to `batch` of them per call.  The host keeps only the tree.

Branching variables: the placement binaries c[f,j] and the node binaries n[j] of the engine's
integer vector (include/neptune_lp.h).  moved_from / moved_to / allocated / deallocated follow
from c — with c integral their LP optimum is integral — and are never branched on.

Multi-GPU: with a communicator (`core/engine/comm.py`, one rank per GPU) every
rank runs the same search redundantly until the open-node frontier holds `world * batch` nodes,
then keeps the frontier nodes whose canonical position is its rank modulo `world` and searches
those subtrees alone.  Per batch the ranks exchange the incumbent value (all-reduce MIN, 8 B) and
their open-node counts (all-reduce SUM, termination); at the end the owner of the best incumbent
(lowest rank on ties) broadcasts its placement.  No collective runs inside an LP.

Warm starts: with `lp.max_batch >= 2 * batch + 1` (and an engine with nep_lp_copy_state) every
node LP after the root starts from its parent's final PDHG state when the parent is still resident
— batches alternate between the two halves of the slots, so the previous batch's nodes (the
parents of the children best-first pops next) stay on the device — else from the root's state,
kept in the last slot (SCIP warm-starts its node LPs from the parent basis the same way).  The
engine floors a warm-started LP's primal weight at 2x the parent's.

Exactness:
  * a node's value is the engine's certified Lagrangian bound, a valid lower bound even when PDHG
    stopped at its iteration limit, so pruning never discards the optimum;
  * an incumbent is only ever a *leaf* — every c and n fixed — whose LP the engine certified
    optimal; with c and n fixed, that LP's optimum is the MIP objective of the placement;
  * the search ends with the queue empty: the incumbent is optimal within `gap` (relative).
"""
import heapq
import itertools
import math
import time

import numpy as np

from .comm import LocalComm
from .lp import LP_CUTOFF, LP_INFEASIBLE, LP_OPTIMAL

OPTIMAL, INFEASIBLE, LIMIT = "OPTIMAL", "INFEASIBLE", "LIMIT"


class BnBResult:
    """Outcome of one search: status, incumbent objective / integer vector / dense routing."""

    def __init__(self):
        self.status = INFEASIBLE
        self.objective = None
        self.z = None            # engine integer vector of the incumbent
        self.x = None            # routing x[i][f][j] of the incumbent (float32)
        self.bound = -math.inf   # best proven lower bound
        self.nodes = 0
        self.leaves = 0
        self.lps = 0
        self.lp_iterations = 0
        self.unresolved = 0      # leaves whose LP hit the iteration limit (not used as incumbents)
        self.seconds = 0.0

    def as_dict(self):
        return {k: getattr(self, k) for k in ("status", "objective", "bound", "nodes", "leaves", "lps",
                                              "lp_iterations", "unresolved", "seconds")}


class BranchAndBound:
    """Best-first B&B with batched node LPs.

    lp            core.engine.lp.LPModel of the step model (max_batch >= batch)
    workload      W [F, N] (to weigh the pooled zero-workload routing rows when computing flows)
    fn_mem/node_mem  memory data for the rounding heuristic's capacity check (C3)
    upper_bound   a-priori bound on any feasible objective: LPs whose Lagrangian exceeds it are
                  stopped early (infeasible nodes have an unbounded Lagrangian)
    """

    def __init__(self, lp, workload, fn_mem, node_mem, batch=16, tol=1e-7, gap=1e-6, max_iters=5000,
                 node_limit=20000, time_limit=None, upper_bound=math.inf, flow_tol=1e-4, log=None, comm=None,
                 warm=True, root_max_iters=200000):
        self.lp = lp
        self.N, self.F = lp.N, lp.F
        L = lp.layout()
        self.c0, self.c1 = L["c"]
        self.n_range = L["n"]
        W = np.asarray(workload, np.float64).reshape(self.F, self.N)
        self.zero_src = (W == 0).sum(axis=1).astype(np.float64)
        self.fn_mem = np.asarray(fn_mem, np.float64).reshape(self.F)
        self.node_mem = np.asarray(node_mem, np.float64).reshape(self.N)
        self.batch = min(int(batch), lp.max_batch)
        self.warm = bool(warm) and hasattr(lp, "copy_state") and lp.max_batch >= 2 * self.batch + 1
        self.root_slot = lp.max_batch - 1
        self.slot_gen = [0] * lp.max_batch     # bumped whenever a slot takes a new LP
        # node LPs stop at max_iters (their Lagrangian bound stays valid for pruning; a leaf only
        # becomes an incumbent when certified); the root, solved cold, gets root_max_iters
        self.tol, self.gap, self.max_iters = tol, gap, max_iters
        self.root_max_iters = max(max_iters, root_max_iters)
        self.node_limit, self.time_limit = node_limit, time_limit
        self.ub0 = upper_bound
        self.flow_tol = flow_tol
        self.log = log or (lambda *_: None)
        self.comm = comm or LocalComm()
        self.branch_vars = list(range(self.c0, self.c1))
        if self.n_range is not None:
            self.branch_vars += list(range(*self.n_range))
        self._nb = len(self.branch_vars)

    # ---------------------------------------------------------------------------------------
    def _gap_abs(self, inc):
        return self.gap * max(1.0, abs(inc)) if math.isfinite(inc) else 0.0

    def _flows(self, slot):
        """flow[f, j] = sum over sources of x[i, f, j] (pooled rows weighted by their size)."""
        xb, rf, rs = self.lp.rows(slot)
        w = np.where(rs >= 0, 1.0, self.zero_src[rf])
        flow = np.zeros((self.F, self.N))
        np.add.at(flow, rf, w[:, None] * xb.astype(np.float64))
        return flow

    def _complete(self, fix):
        return len(fix) >= self._nb

    def _round(self, fix, flow):
        """Heuristic completion of a node: c = 1 where fixed to 1 or carrying flow, n = any c.
        Returns a full fixing dict, or None when it is visibly infeasible."""
        F, N, c0 = self.F, self.N, self.c0
        c = np.zeros(F * N)
        free = np.ones(F * N, bool)
        for k, v in fix.items():
            if c0 <= k < self.c1:
                c[k - c0] = v
                free[k - c0] = False
        c[free & (flow.ravel() > self.flow_tol)] = 1.0
        cm = c.reshape(F, N)
        if (cm.sum(axis=1) < 1).any():
            return None
        if ((self.fn_mem[:, None] * cm).sum(axis=0) > self.node_mem + 1e-9).any():
            return None
        leaf = {c0 + k: float(c[k]) for k in range(F * N)}
        if self.n_range is not None:
            n0 = self.n_range[0]
            nv = (cm.sum(axis=0) >= 1).astype(np.float64)
            for j in range(N):
                if fix.get(n0 + j, nv[j]) != nv[j]:
                    return None
                leaf[n0 + j] = float(nv[j])
        return leaf

    def _branch_var(self, fix, z, flow):
        """n[j] receiving flow (largest inflow), then c[f,j] carrying flow (largest), then any free
        n / c by LP value.  None when every branching variable is fixed."""
        F, N, c0 = self.F, self.N, self.c0
        if self.n_range is not None:
            n0 = self.n_range[0]
            inflow = flow.sum(axis=0)
            cand = [j for j in range(N) if (n0 + j) not in fix and inflow[j] > self.flow_tol]
            if cand:
                return n0 + max(cand, key=lambda j: (inflow[j], -j))
        fl = flow.ravel()
        cand = [k for k in range(F * N) if (c0 + k) not in fix and fl[k] > self.flow_tol]
        if cand:
            return c0 + max(cand, key=lambda k: (fl[k], -k))
        free = [v for v in self.branch_vars if v not in fix]
        if not free:
            return None
        return max(free, key=lambda v: (z[v], -v))

    def _place(self, batch, half, root_ready):
        """Slots of this batch's LPs and whether they start warm.  Cold: slots 0..B-1.  Warm: the
        half of the slots the previous batch did not use; each LP starts from its parent's state if
        that is still resident in the other half, else from the root's."""
        B = len(batch)
        if not (self.warm and root_ready):
            slots = np.arange(B, dtype=np.int32)
            for s in slots:
                self.slot_gen[s] += 1
            return slots, False
        base = half * self.batch
        slots = np.arange(base, base + B, dtype=np.int32)
        for b, (_, _, _, pref) in enumerate(batch):
            src = self.root_slot
            if pref is not None:
                ps, pg = pref
                if self.slot_gen[ps] == pg and not (base <= ps < base + self.batch):
                    src = ps
            self.lp.copy_state(src, int(slots[b]))
        for s in slots:
            self.slot_gen[s] += 1
        return slots, True

    # ---------------------------------------------------------------------------------------
    def solve(self):
        t0 = time.time()
        res = BnBResult()
        lp, n_int = self.lp, self.lp.n_int
        inc = math.inf
        seq = itertools.count()
        # (bound, -depth, seq, fixings, is_leaf, parent) with parent = (slot, generation) or None
        heap = [(-math.inf, 0, next(seq), {}, False, None)]
        pending_leaves = []                              # (fixings, parent)
        half = 0
        root_ready = False
        seen_leaves = set()
        limit_hit = False
        comm = self.comm
        sharded = comm.world == 1
        while True:
            if not sharded and len(heap) >= comm.world * self.batch:
                # deal the (identical on every rank) frontier: canonical order, round robin
                heap.sort()
                heap = [h for i, h in enumerate(heap) if i % comm.world == comm.rank]
                heapq.heapify(heap)
                pending_leaves = [lf for i, lf in enumerate(pending_leaves) if i % comm.world == comm.rank]
                sharded = True
            if comm.world > 1 and sharded:
                inc = comm.min(inc)
                if comm.sum(len(heap) + len(pending_leaves)) == 0:
                    break
            elif not (heap or pending_leaves):
                break
            if res.nodes >= self.node_limit or (self.time_limit and time.time() - t0 > self.time_limit):
                limit_hit = True
                if comm.world > 1 and sharded:
                    heap, pending_leaves = [], []
                    continue
                break
            batch = []
            while pending_leaves and len(batch) < self.batch:
                leaf, pref = pending_leaves.pop()
                batch.append((-math.inf, leaf, True, pref))
            while heap and len(batch) < self.batch:
                bnd, _, _, fix, is_leaf, pref = heapq.heappop(heap)
                if bnd >= inc - self._gap_abs(inc):
                    continue
                batch.append((bnd, fix, is_leaf, pref))
            if not batch:
                continue
            B = len(batch)
            slots, warm = self._place(batch, half, root_ready)
            half ^= 1
            lb = np.full((B, n_int), -np.inf)
            ub = np.full((B, n_int), np.inf)
            for b, (_, fix, _, _) in enumerate(batch):
                if fix:
                    idx = np.fromiter(fix.keys(), np.int64, len(fix))
                    val = np.fromiter(fix.values(), np.float64, len(fix))
                    lb[b, idx] = val
                    ub[b, idx] = val
            cutoff = min(inc, self.ub0)
            is_root = res.lps == 0
            r = lp.solve(slots, lb, ub, tol=self.tol, max_iters=self.root_max_iters if is_root else self.max_iters,
                         cutoff=cutoff if math.isfinite(cutoff) else math.inf, warm_start=warm)
            res.lps += B
            res.lp_iterations += int(r["iters"].sum())
            for b, (pbound, fix, is_leaf, _) in enumerate(batch):
                slot = int(slots[b])
                st = int(r["status"][b])
                if self.warm and not fix and not root_ready and st not in (LP_INFEASIBLE, LP_CUTOFF):
                    lp.copy_state(slot, self.root_slot)   # every later node can start from the root
                    root_ready = True
                if st in (LP_INFEASIBLE, LP_CUTOFF):
                    continue
                bound = max(pbound, float(r["obj"][b]))
                if is_leaf:
                    res.leaves += 1
                    if st != LP_OPTIMAL:
                        res.unresolved += 1
                        continue
                    val = float(r["primal_obj"][b])
                    if val < inc - self._gap_abs(inc):
                        inc = val
                        res.objective = val
                        res.z, res.x = lp.solution(slot, dense_x=True)
                        self.log(f"incumbent {val:.10g} (lps {res.lps}, nodes {res.nodes})")
                    continue
                if bound >= inc - self._gap_abs(inc):
                    continue
                res.nodes += 1
                z, _ = lp.solution(slot, dense_x=False)
                flow = self._flows(slot)
                me = (slot, self.slot_gen[slot])
                leaf = self._round(fix, flow)
                if leaf is not None:
                    key = tuple(sorted(k for k, v in leaf.items() if v > 0.5))
                    if key not in seen_leaves:
                        seen_leaves.add(key)
                        pending_leaves.append((leaf, me))
                var = self._branch_var(fix, z, flow)
                if var is None:
                    continue
                for v in (1.0, 0.0):
                    child = dict(fix)
                    child[var] = v
                    heapq.heappush(heap, (bound, -len(child), next(seq), child, self._complete(child), me))
        if heap:
            res.bound = min(min(h[0] for h in heap), inc)
        else:
            res.bound = inc
        if comm.world > 1:
            res.bound = comm.min(res.bound)
            limit_hit = comm.sum(int(limit_hit)) > 0
            # the owner of the best incumbent (lowest rank on ties) broadcasts the placement
            mine = res.objective is not None and res.objective <= inc
            owner = int(comm.min(comm.rank if mine else comm.world))
            if owner < comm.world:
                nz = self.lp.n_int
                z = res.z if mine and comm.rank == owner else np.zeros(nz)
                x = res.x if mine and comm.rank == owner else np.zeros((self.N, self.F, self.N), np.float32)
                res.z = comm.bcast(np.asarray(z, np.float64), owner)
                res.x = comm.bcast(np.asarray(x, np.float32), owner)
                res.objective = inc
            res.nodes = comm.sum(res.nodes)
            res.lps = comm.sum(res.lps)
        if res.objective is None:
            res.status = LIMIT if limit_hit else INFEASIBLE
        else:
            res.status = LIMIT if limit_hit else OPTIMAL
        res.seconds = time.time() - t0
        return res
