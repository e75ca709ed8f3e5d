"""Streaming best-first branch-and-bound over the MI355X LP engine.

This is the tree search SCIP runs inside `pywraplp.Solver.Solve()` (reference
`core/solvers/solver.py:35-40`) on the NEPTUNE step models, rebuilt around the engine's streaming
node-LP API (`nep_lp_submit` / `nep_lp_advance`, include/neptune_lp.h): up to `batch` node LPs
iterate on the device at once and a slot whose LP finishes takes the next open node at once, so no
slot waits for the slowest LP of a batch.  Per finished node only small results cross PCIe: its
status / bound, and the per-(function, destination) flows reduced on the device
(`nep_lp_get_flows`, F x N floats) — the host keeps only the tree.

Branching variables: the placement binaries c[f,j] and the node binaries n[j] of the engine's
integer vector.  moved_from / moved_to / allocated / deallocated follow from c — with c integral
their LP optimum is integral — and are never branched on.

Exactness:
  * a node's value is the engine's Lagrangian bound, a valid lower bound even when its LP stopped
    at the iteration limit, so pruning never discards the optimum;
  * an incumbent is only a *leaf* (every c and n fixed) whose LP the engine certified: the
    certificate's repaired primal point is feasible, so its value is attained;
  * a leaf whose LP stops uncertified is re-solved once with the root's iteration budget; if it
    still does not certify its bound stays in `res.bound` and the search reports LIMIT (never
    OPTIMAL or INFEASIBLE) while that bound is below the incumbent;
  * the search ends with no open node: the incumbent is optimal within `gap` (relative).

Warm starts: every node LP after the root starts from its parent's final PDHG state when the
parent's slot still holds it (slots are reused least-recently-finished first), else from the
root's, kept in a reserved slot (SCIP warm-starts its node LPs from the parent basis the same way).

Strengthened bounds (round 4): with `bound_lp` (an LPModel of the facility relaxation,
NEP_RELAX_FACILITY: x[i,f,j] <= c[f,j] and c[f,j] <= n[j] in place of the big-M pairs, valid for every
integral placement) the branching nodes' LPs run on that model and give the search its bounds, flows and
rounding input; leaves (every c and n fixed) still run on the reference model `lp`, whose certified LP is
the incumbent (its point is feasible for the reference's rows, C2's eps floors included).  The two models
iterate on their own HIP streams side by side; leaves warm-start from the reference root LP's state,
solved beside the first bound LPs.

Multi-GPU (core/engine/comm.py, one rank per GPU): every rank runs the same search
redundantly until the open-node frontier holds `world * batch` nodes, then keeps the frontier nodes
whose canonical position is its rank modulo `world` and searches those subtrees alone.  Every loop
the ranks agree (all-reduce) on the incumbent value (MIN), on stopping (time / node limit of ANY rank)
and on termination (open + in-flight node count, SUM); at the end the owner of the best incumbent
(lowest rank on ties) broadcasts its placement.  No collective runs inside an LP.
"""
import heapq
import itertools
import math
import os
import time
from collections import deque

import numpy as np

from .comm import LocalComm
from .lp import LP_BOUND, LP_CUTOFF, LP_INFEASIBLE, LP_ITERATION_LIMIT, LP_OPTIMAL, round_leaf, round_leaves

OPTIMAL, INFEASIBLE, LIMIT = "OPTIMAL", "INFEASIBLE", "LIMIT"
_STATUS_NAME = {LP_OPTIMAL: "certified", LP_ITERATION_LIMIT: "limit", LP_INFEASIBLE: "infeasible",
                LP_CUTOFF: "cutoff", LP_BOUND: "bound"}
NODE, LEAF, RETRY, REFROOT = 0, 1, 2, 3
# step-2 searches on the native tree (NEP_BNB_STEP2 overrides)
STEP2_NATIVE_DEFAULT = "1"
_KIND_NAME = {NODE: "node", LEAF: "leaf", RETRY: "retry", REFROOT: "refroot"}


class BnBResult:
    """Outcome of one search: status, incumbent objective / integer vector / dense routing."""

    def __init__(self):
        self.status = INFEASIBLE
        self.objective = None
        self.z = None            # engine integer vector of the incumbent
        self.x = None            # routing x[i][f][j] of the incumbent: core.engine.routing.SparseRouting (the
                                 # device-compacted entries, fetched once at the end; never the dense matrix)
        self.bound = -math.inf   # best proven lower bound
        self.nodes = 0           # branched (non-leaf) nodes whose LP finished
        self.leaves = 0
        self.lps = 0             # node LPs submitted (presolve-infeasible ones included)
        self.certified = 0       # node LPs the engine certified optimal
        self.lp_iterations = 0
        self.unresolved = 0      # leaves still uncertified after their retry
        self.seconds = 0.0
        self.incumbent_slot = None
        self.polished = False    # the incumbent's LP was re-solved at the polish tolerance
        self.repaired = None     # the CPU repair of the returned routing succeeded (None: not run)
        self.heuristic_incumbents = 0   # incumbents taken from a checked heuristic point (no LP behind them)
        self.routing_warm = 0           # leaves warm-started with their branching node's routing (two models)
        # node-LP mix: finished LPs per engine status (+ presolve-infeasible submits) and their iterations
        self.lp_status = {"certified": 0, "bound": 0, "limit": 0, "infeasible": 0, "cutoff": 0, "numerical": 0,
                          "presolve_infeasible": 0}
        self.lp_status_kind = {k: dict.fromkeys(self.lp_status, 0) for k in ("node", "leaf", "retry", "refroot")}
        self.lp_iters = []
        self.drained = 0         # LPs still iterating at a stop decision (stopped at their next check)
        # wall seconds by phase: device waits in advance, host work per finished LP, submits (incl.
        # warm-start copies), the drain after a stop, the end (routing fetch, polish, repair)
        self.timing = dict.fromkeys(("advance", "finish", "submit", "drain", "end", "primal"), 0.0)
        self.timing["root"] = 0.0       # wall seconds until the root LP finished (it iterates alone)
        self.split_hash = None          # sharded search: crc32 of the frontier every rank dealt (must agree)
        self.rebalanced = 0             # open nodes this rank received from another rank
        self.advance_calls = 0
        self.inflight_sum = 0           # LPs in flight summed over the advance calls (mean: / advance_calls)
        self.native = False             # the search ran on the native tree (csrc/nep_bnb.cpp)
        self.strong = None              # (native, branching 2) strong-branching probe counts

    def as_dict(self):
        d = {k: getattr(self, k) for k in ("status", "objective", "bound", "nodes", "leaves", "lps", "certified",
                                           "lp_iterations", "unresolved", "seconds", "polished", "repaired",
                                           "lp_status", "lp_status_kind", "drained", "timing",
                                           "heuristic_incumbents", "routing_warm", "native", "strong")}
        d["inflight_mean"] = self.inflight_sum / max(1, self.advance_calls)
        d["resolved"] = sum(v for k, v in self.lp_status.items() if k not in ("limit", "numerical"))
        it = np.asarray(self.lp_iters, np.float64)
        d["lp_iters_p50_p90_p99_max"] = ([float(v) for v in np.percentile(it, [50, 90, 99, 100])] if it.size else None)
        return d


class _Node:
    __slots__ = ("bound", "idx", "val", "kind", "parent", "depth", "nid")

    def __init__(self, bound, idx, val, kind, parent, depth):
        # parent: (engine, slot, slot generation, parent's id) of the LP whose state may warm-start this one
        self.bound, self.idx, self.val, self.kind, self.parent, self.depth = bound, idx, val, kind, parent, depth
        self.nid = -1            # submission order (the trace's id)


class _Engine:
    """One LP model's slots: a free list of working slots, a reserved slot for its root LP's state (the
    warm-start source of nodes whose parent's state is gone) and, on the leaf engine, one for the incumbent's;
    per-slot generations tell a parent's state from a later occupant's."""

    def __init__(self, lp, reserve, name):
        self.lp, self.name = lp, name
        self.reserved = reserve if lp.max_batch > reserve else 0
        self.root_slot = lp.max_batch - 1
        self.inc_slot = lp.max_batch - 2
        self.gen = [0] * lp.max_batch
        self.free = deque(range(lp.max_batch - self.reserved))
        self.root_ready = False
        self.root_state = False      # root_slot holds the root LP's final state (a warm-start source)
        self.inflight = 0


class BranchAndBound:
    """Streaming best-first B&B.

    lp            core.engine.lp.LPModel of the step model (max_batch >= batch + 2: `batch` working
                  slots, one for the root's state, one for the incumbent's)
    bound_lp      optional LPModel of the strengthened relaxation (NEP_RELAX_FACILITY) the branching nodes
                  are bounded with (max_batch >= batch + 1: one slot for its root's state); None: every node
                  LP runs on `lp`
    workload      W [F, N] (unused since the flows are reduced on the device; kept for the API)
    fn_mem/node_mem  memory data for the rounding heuristic's capacity check (C3)
    upper_bound   a-priori bound on any feasible objective: LPs whose Lagrangian exceeds it stop early
    """

    def __init__(self, lp, workload, fn_mem, node_mem, batch=16, tol=1e-7, gap=1e-6, max_iters=5000,
                 node_limit=20000, time_limit=None, upper_bound=math.inf, flow_tol=1e-4, log=None, comm=None,
                 warm=True, root_max_iters=200000, check_every=12, polish_tol=1e-8, polish_iters=20000,
                 seed_leaves=None, integer_bound=None, improve=None, repair=None, node_bound_res=1e-2,
                 retry_res=math.inf, unit_flow_leaves=True, node_max_iters=None, bound_lp=None, bound_gap=1e-4,
                 trace=None, rebalance_every=8, primal=None, primal_every=0,
                 leaf_routing_warm=False, root_check_every=64, objective_integral=False, warm_weight_ref=0.0,
                 native=None, step2_native=None, branching=0, strong_cands=8, strong_rel=2, strong_iters=256):
        self.lp = lp
        self.two = bound_lp is not None
        self.N, self.F = lp.N, lp.F
        L = lp.layout()
        self.c0, self.c1 = L["c"]
        self.n_range = L["n"]
        self.fn_mem = np.asarray(fn_mem, np.float64).reshape(self.F)
        self.node_mem = np.asarray(node_mem, np.float64).reshape(self.N)
        self.reserved = 2 if lp.max_batch >= 3 else 0
        self.batch = max(1, min(int(batch), lp.max_batch - self.reserved))
        # (the bound model: its slots beyond `batch` + its root's park finished parents' states)
        self.batch_b = max(1, min(int(batch), bound_lp.max_batch - 1)) if bound_lp is not None else self.batch
        self.warm = bool(warm) and self.reserved == 2 and (bound_lp is None or bound_lp.max_batch >= 2)
        self.bound_lp = bound_lp
        # the bound model's LPs stop once their own gap (repaired point vs best bound) is within bound_gap:
        # a node needs its bound, which is valid at any dual point; the leaves keep the certificate tolerance
        self.bound_gap = bound_gap
        # trace: a list that receives one entry per submitted node LP (_trace_entry), or None
        self.trace = trace
        # sharded search: every rebalance_every loops, ranks with an empty frontier take open nodes from the
        # fullest ones (_rebalance; 0: never)
        self.rebalance_every = rebalance_every
        # primal(idx, val, z, flow) -> [(idx, val[, sol])]: leaves completing a branching node's fixings, built
        # from its LP (z, flow) with the instance's data (core/engine/heuristics.py); sol, when given, is a
        # feasible point of that leaf checked by the caller ({"objective", "z", "row", "dst", "val"}: a direct
        # incumbent before any LP runs on the leaf, whose LP is queued too); run at the root and, with
        # primal_every > 0, on every primal_every-th branched node (0: the root only — with the facility
        # relaxation's bounds the nodes' own rounding leaves find the same incumbents at 256x128 / 512x256, and
        # the greedy costs ~2 s per call at 512x256)
        self.primal = primal
        self.primal_every = max(0, int(primal_every))
        # two models: a rounding leaf starts from the reference root's state with the routing x of the
        # branching node it was rounded from (nep_lp_copy_routing) while that node's slot still holds it.
        # Off by default: 256x128 / 512x256, 20 s, measured no better
        self.leaf_routing_warm = bool(leaf_routing_warm)
        # the roots (which run alone on their model, tens of thousands of iterations) take a certificate
        # check every root_check_every iterations instead of check_every: a 1-slot certificate launch costs
        # ~3 plain ones (bench.py's root uses 64 as well)
        self.root_check_every = int(root_check_every) if root_check_every else check_every
        self.root_slot = lp.max_batch - 1
        self.inc_slot = lp.max_batch - 2
        self.tol, self.gap, self.max_iters = tol, gap, max_iters
        # every integral point has an integral objective (step 2's disruption objective, objectives.py:55-63;
        # step-1 MinUtilization's node count): a node whose valid bound exceeds incumbent - 1 holds no better
        # point, so it is pruned (SCIP's objective-integrality pruning)
        # (a number: the objective's integral unit, e.g. alpha / N for MinDelayAndUtilization without workload)
        self.objective_integral = bool(objective_integral)
        self.objective_unit = (1.0 if objective_integral is True or not isinstance(objective_integral, (int, float))
                               else float(objective_integral)) if objective_integral else 0.0
        # warm_weight_ref > 0: warm-started node LPs take their PDHG primal weight in [2, 4] x (warm_weight_ref x
        # the model's cold-start weight omega0) instead of [2, 4] x their parent's final weight, which ratchets up
        # along a lineage (nep_lp_set_reference_weight; step 1 at 512x256: replay 7.5 -> 12.2 certified LP/s,
        # independent of the root's chaotic final weight; DESIGN.md §4 "Warm-start primal weight").  0 (default):
        # parent-relative — the step-2 models keep it (a 64x32 delete node LP stalls under the step-1 band)
        self.warm_weight_ref = float(warm_weight_ref or 0.0)
        # native tree search (csrc/nep_bnb.cpp, nep_bnb_*): the single-rank search without per-node Python
        # callbacks runs its whole loop in the engine library (None: whenever eligible; NEP_BNB_PYTHON=1 keeps
        # this module's loop, for A/B)
        self.native = native
        # (create, node_cap, old allocation [F*N]): integer_bound is step 2's closed form, which the native tree
        # evaluates itself (NeptuneStep2Base.native_bound); improve then runs on NEP_BNB_INCUMBENT events
        self.step2_native = step2_native
        # branching rule of the native tree: 0 = n by largest inflow, then c by largest flow (this module's loop);
        # 1 = pseudo-cost branching (product score over fractional n / c, csrc/nep_bnb.cpp branch_var_pc); 2 = reliability
        # branching: pseudo-costs, with strong-branching probe LPs (strong_iters iterations, both children of the
        # strong_cands best candidates) while a candidate's pseudo-costs rest on fewer than strong_rel observations
        self.branching = int(branching)
        self.strong_cands, self.strong_rel, self.strong_iters = int(strong_cands), int(strong_rel), int(strong_iters)
        # (the leaf / reference model only — the model whose node LPs the replay measured; the facility relaxation
        # keeps the parent-relative band: 256x128 / 20 s gap 0.51 % with it, 0.82 % with the band on both)
        for m_ in (lp,):
            if m_ is not None and hasattr(m_, "set_reference_weight"):
                m_.set_reference_weight(self.warm_weight_ref * m_.info.primal_weight0 if self.warm_weight_ref > 0 else 0.0)
        self.root_max_iters = max(max_iters, root_max_iters)
        self.check_every = check_every
        # the final incumbent's LP is re-solved (warm, from its own state) at polish_tol, so the
        # returned routing also meets the reference's absolute checker tolerances
        # (efttc/utils/constraints_step1.py:68-78: CPU <= cores + 1e-6)
        self.polish_tol, self.polish_iters = polish_tol, polish_iters
        # seed_leaves: [(idx, val)] placements queued as leaves after the root (primal starts);
        # integer_bound(idx, val): a model-specific lower bound valid for every integral completion of
        # a node's fixings (+inf: none); a node's bound is the larger of it and its parent LP's
        self.seed_leaves = list(seed_leaves or [])
        self.integer_bound = integer_bound
        # improve(idx, val, value) -> [(idx, val)]: neighbour leaves of each new incumbent (local search)
        self.improve = improve
        # repair(x, z) -> (x', objective change, ok): the returned routing moved within its placement so
        # it meets the reference checker's absolute CPU tolerance (core.engine.routing.repair_cpu)
        self.repair = repair
        # branching nodes (not leaves, not the root) stop once their bound has converged, with the repaired
        # point's residual <= node_bound_res (engine status LP_BOUND): a node branches on its bound, which
        # is valid at any dual point, so it need not iterate on to primal feasibility at tol (0: off)
        self.node_bound_res = node_bound_res
        # an uncertified leaf is re-solved with the root budget only when its repaired point's residual
        # at the node-LP limit is <= retry_res (a leaf the rounding made CPU-infeasible ends far above it
        # and would burn the root budget); otherwise its bound stays as an unresolved one
        self.retry_res = retry_res
        # iteration limit of branching nodes (their bound is valid wherever they stop); leaves keep max_iters
        self.node_max_iters = int(node_max_iters) if node_max_iters else max_iters
        # rounding leaves per branched node: fewest openings, every (f, j) with flow, and (unit_flow_leaves)
        # every (f, j) with a unit of flow (_round's min_flow)
        self.round_modes = ((False, None), (True, None)) + (((True, 1.0 - 1e-6),) if unit_flow_leaves else ())
        self.node_limit, self.time_limit = node_limit, time_limit
        self.ub0 = upper_bound
        self.flow_tol = flow_tol
        self.log = log or (lambda *_: None)
        self.comm = comm or LocalComm()
        nb = self.c1 - self.c0 + (0 if self.n_range is None else self.n_range[1] - self.n_range[0])
        self._nb = nb

    # ---------------------------------------------------------------------------------------
    def _gap_abs(self, inc):
        if not math.isfinite(inc):
            return 0.0
        g = self.gap * max(1.0, abs(inc))
        if self.objective_integral:
            # bound >= inc - unit + delta prunes; delta covers the fp64 error of a Lagrangian bound of this size
            u = self.objective_unit if self.objective_unit > 0 else 1.0
            g = max(g, u * (1.0 - min(0.5, 1e-6 + 1e-9 * abs(inc) / u)))
        return g

    def _ibound(self, idx, val):
        return -math.inf if self.integer_bound is None else float(self.integer_bound(idx, val))

    def _fixed(self, node):
        fx = np.zeros(self.lp.n_int, bool)
        fx[node.idx] = True
        return fx

    def _round_all(self, node, flow, zc):
        """_round for every rounding mode (self.round_modes) of one node in one native call."""
        F, N, c0, c1 = self.F, self.N, self.c0, self.c1
        fixed = np.full(F * N, -1.0)
        sel = (node.idx >= c0) & (node.idx < c1)
        fixed[node.idx[sel] - c0] = node.val[sel]
        nfix = None
        if self.n_range is not None:
            n0, n1 = self.n_range
            nfix = np.full(N, -1.0)
            seln = (node.idx >= n0) & (node.idx < n1)
            nfix[node.idx[seln] - n0] = node.val[seln]
        modes = [(bf, self.flow_tol if mf is None else mf) for bf, mf in self.round_modes]
        out = []
        for r in round_leaves(fixed.reshape(F, N), nfix, np.asarray(flow).reshape(F, N), zc, self.fn_mem,
                              self.node_mem, modes):
            if r is None:
                out.append(None)
            elif r[1] is None:
                out.append((np.arange(c0, c1), r[0]))
            else:
                out.append((np.concatenate([np.arange(c0, c1), np.arange(*self.n_range)]), np.concatenate(r)))
        return out

    def _round(self, node, flow, zc=None, by_flow=True, min_flow=None):
        """Heuristic completion of a node (a leaf fixing every c and n), or None.

        Memory-aware greedy rounding of the node LP (native: nep_round_leaf, csrc/nep_round.cpp): the fixed
        c stay as fixed; the free c the LP holds at >= 1/2 (zc, the LP's c) are opened first, largest first,
        then the free (f, j) in decreasing order of the flow f sends to j, while node j's memory (C3,
        constraints_step1.py:18-23) has room and n[j] is not fixed to 0; a function left without an open
        destination gets the one with the largest LP c, then flow, that still has room; n[j] = any c[:, j]
        (a node fixed open gets its best-fitting function).  The leaf's LP then re-optimises x.  (Opening
        the LP's near-integral c first is what keeps step 2's placement next to the old allocation: its LP
        c sits at old wherever no flow forces a move.)  by_flow=False skips the flow pass: the fewest
        openings the LP's c allows (a leaf whose x must then fit the CPU rows with those openings only).
        min_flow: the flow pass opens only the (f, j) the LP already sends >= min_flow (an open (f, j) must
        receive >= 1 - eps, C2, so opening a trickle forces a unit of flow onto j's CPU; at 512x256 such
        leaves end CPU-infeasible).  tests/round_ref.py keeps the Python form it was until round 4, and
        tests/test_round_native.py holds the two to the same leaves."""
        F, N, c0, c1 = self.F, self.N, self.c0, self.c1
        fixed = np.full(F * N, -1.0)
        sel = (node.idx >= c0) & (node.idx < c1)
        fixed[node.idx[sel] - c0] = node.val[sel]
        nfix = None
        if self.n_range is not None:
            n0, n1 = self.n_range
            nfix = np.full(N, -1.0)
            seln = (node.idx >= n0) & (node.idx < n1)
            nfix[node.idx[seln] - n0] = node.val[seln]
        thr = self.flow_tol if min_flow is None else min_flow
        out = round_leaf(fixed.reshape(F, N), nfix, np.asarray(flow).reshape(F, N), zc, self.fn_mem, self.node_mem,
                         by_flow, thr)
        if out is None:
            return None
        c, nv = out
        if nv is None:
            return np.arange(c0, c1), c
        return np.concatenate([np.arange(c0, c1), np.arange(*self.n_range)]), np.concatenate([c, nv])

    def _branch_var(self, node, flow, slot, lp=None):
        """n[j] receiving flow (largest inflow), then c[f,j] carrying flow (largest), then any free
        n / c by LP value (ties: lowest index).  None when every branching variable is fixed."""
        fixed = self._fixed(node)
        if self.n_range is not None:
            n0, n1 = self.n_range
            inflow = flow.sum(axis=0).astype(np.float64)
            cand = np.flatnonzero(~fixed[n0:n1] & (inflow > self.flow_tol))
            if cand.size:
                return n0 + int(cand[np.argmax(inflow[cand])])
        fl = flow.ravel().astype(np.float64)
        cand = np.flatnonzero(~fixed[self.c0:self.c1] & (fl > self.flow_tol))
        if cand.size:
            return self.c0 + int(cand[np.argmax(fl[cand])])
        free = np.flatnonzero(~fixed[self.c0:self.c1]) + self.c0
        if self.n_range is not None:
            free = np.concatenate([free, np.flatnonzero(~fixed[self.n_range[0]:self.n_range[1]]) + self.n_range[0]])
        if free.size == 0:
            return None
        z, _ = (lp or self.lp).solution(slot, dense_x=False)
        zf = z[free]
        return int(free[np.argmax(zf)])

    # ---------------------------------------------------------------------------------------
    def _submit(self, items, inc):
        """items: [(engine, slot, node)].  One nep_lp_submit per (engine, warm, iteration budget) group."""
        groups = {}
        copies = {}
        cross = []               # (leaf slot, branching-node slot of the bound model): routing warm starts
        cutoff = min(inc, self.ub0)
        for eng, slot, node in items:
            warm, src = False, None
            if self.warm and eng.root_ready:
                # (the root slot holds a state only when the root LP ended with one: an infeasible / cut-off
                # root leaves it empty, and its nodes then start cold unless their parent's state is resident)
                src = eng.root_slot if eng.root_state else None
                if node.parent is not None:
                    pe, ps, pg = node.parent[:3]
                    if pe is eng and eng.gen[ps] == pg:
                        src = ps
                if src is not None:
                    if src != slot:
                        copies.setdefault(eng.name, (eng, []))[1].append((src, slot))
                    warm = True
                if (self.two and self.leaf_routing_warm and node.kind == LEAF and eng is self.L
                        and node.parent is not None and node.parent[0] is self.B
                        and self.B.gen[node.parent[1]] == node.parent[2]):
                    cross.append((slot, node.parent[1]))
            budget = (self.root_max_iters if (node.kind in (RETRY, REFROOT) or not eng.root_ready)
                      else (self.node_max_iters if node.kind == NODE else self.max_iters))
            # (the bound model's root is a branching node like the others: it stops once its bound converged)
            bres = self.node_bound_res if (node.kind == NODE and (eng.root_ready or self.two)) else 0.0
            ce = self.root_check_every if (node.kind == REFROOT or not eng.root_ready) else self.check_every
            groups.setdefault((eng.name, warm, budget, bres, ce), (eng, []))[1].append((slot, node))
            node.nid = next(self.nid_seq)
            if self.trace is not None:
                self.trace.append(self._trace_entry(eng, node, src if warm else None, budget, bres, cutoff))
        # warm-start copies: a slot that is both a parent state (source) and a new node's slot
        # (destination) is read before it is overwritten; a cycle falls back to the root's state.  The leaf
        # model's copies run first, then the routing copies from the bound model's node slots (before that
        # model's own copies may overwrite them)
        order = sorted(copies.values(), key=lambda ec: 0 if ec[0] is self.L else 1)
        done_cross = not cross
        for eng, cps in order:
            if not done_cross and eng is not self.L:
                self._copy_cross(cross)
                done_cross = True
            while cps:
                srcs = {c[0] for c in cps}
                k = next((i for i, (_, d) in enumerate(cps) if d not in srcs), None)
                if k is None:
                    src, dst = cps[0]
                    cps[0] = (eng.root_slot, dst)
                    continue
                src, dst = cps.pop(k)
                eng.lp.copy_state(src, dst)
        if not done_cross:
            self._copy_cross(cross)
        for (_, warm, budget, bres, ce), (eng, its) in groups.items():
            n_int = eng.lp.n_int
            slots = np.array([s for s, _ in its], np.int32)
            lb = np.full((len(its), n_int), -np.inf)
            ub = np.full((len(its), n_int), np.inf)
            for b, (_, node) in enumerate(its):
                lb[b, node.idx] = node.val
                ub[b, node.idx] = node.val
            gap_tol = self.bound_gap if (self.two and eng is self.B) else 0.0
            st = eng.lp.submit(slots, lb, ub, tol=self.tol, cutoff=cutoff if math.isfinite(cutoff) else math.inf,
                               max_iters=budget, check_every=ce, warm_start=warm, bound_res=bres,
                               gap_tol=gap_tol)
            for b, (slot, node) in enumerate(its):
                eng.gen[slot] += 1
                self.res.lps += 1
                if int(st[b]) == LP_INFEASIBLE:
                    self.res.lp_status["presolve_infeasible"] += 1
                    self.res.lp_status_kind[_KIND_NAME[node.kind]]["presolve_infeasible"] += 1
                    eng.free.append(slot)
                    if node.kind == REFROOT:
                        # the reference root proven infeasible: every leaf (a sub-box of it) is infeasible too.
                        # Mark its engine ready (without a root state) so the loop does not wait for it forever
                        eng.root_ready = True
                else:
                    self.inflight[(eng.name, slot)] = node
                    eng.inflight += 1

    def _finish(self, eng, slot, node, st, obj, pobj, iters, inc, pre=None):
        """Process one finished node LP (of engine `eng`); returns the (possibly improved) incumbent value.
        pre: (flows F x N, z_int) when the caller already read them (one device read per block, _prefetch)."""
        res = self.res
        lp = eng.lp
        eng.inflight -= 1
        res.lp_iterations += iters
        res.lp_iters.append(iters)
        res.lp_status[_STATUS_NAME.get(st, "numerical")] += 1
        res.lp_status_kind[_KIND_NAME[node.kind]][_STATUS_NAME.get(st, "numerical")] += 1
        if node.kind == REFROOT:
            # the reference root LP: its state warm-starts the leaves (their LPs run on this model)
            if self.warm and st not in (LP_INFEASIBLE, LP_CUTOFF):
                lp.copy_state(slot, eng.root_slot)
                eng.root_state = True
            eng.root_ready = True
            eng.free.append(slot)
            return inc
        if st == LP_OPTIMAL:
            res.certified += 1
        if not eng.root_ready and node.depth == 0 and node.kind == NODE:
            res.timing["root"] = time.time() - self.t0
            if self.warm and st not in (LP_INFEASIBLE, LP_CUTOFF):
                lp.copy_state(slot, eng.root_slot)   # every later node can start from the root
                eng.root_state = True
            eng.root_ready = True
            me0 = (eng, slot, eng.gen[slot], node.nid)
            for idx, val in self.seed_leaves:
                idx, val = np.asarray(idx), np.asarray(val, np.float64)
                lb = self._ibound(idx, val)
                if lb < math.inf:
                    key = np.packbits(val > 0.5).tobytes()
                    if key not in self.seen_leaves:
                        self.seen_leaves.add(key)
                        self.pending.append(_Node(lb, idx, val, LEAF, me0, 1))
        if st in (LP_INFEASIBLE, LP_CUTOFF):
            eng.free.append(slot)
            return inc
        bound = max(node.bound, obj)
        if node.kind != NODE:
            res.leaves += 1
            if st == LP_OPTIMAL:
                if pobj < inc - self._gap_abs(inc):
                    inc = pobj
                    res.objective = pobj
                    self.inc_node = node
                    res.z, _ = lp.solution(slot, dense_x=False)
                    if self.warm:
                        lp.copy_state(slot, eng.inc_slot)   # its x is fetched once, at the end
                        res.incumbent_slot = eng.inc_slot
                    else:
                        if res.incumbent_slot is not None and res.incumbent_slot in self.keep:
                            self.keep.discard(res.incumbent_slot)
                            eng.free.append(res.incumbent_slot)
                        res.incumbent_slot = slot
                        self.keep.add(slot)
                    for e in self.engines:
                        e.lp.set_params(self.tol, min(inc, self.ub0))
                    self.log(f"incumbent {pobj:.10g} (lps {res.lps}, nodes {res.nodes})")
                    if self.improve is not None:
                        for idx, val in self.improve(node.idx, node.val, pobj):
                            key = np.packbits(np.asarray(val) > 0.5).tobytes()
                            if key not in self.seen_leaves:
                                self.seen_leaves.add(key)
                                # a neighbour is no descendant of this leaf: its bound is its own
                                self.pending.appendleft(_Node(self._ibound(idx, val), idx,
                                                              np.asarray(val, np.float64), LEAF,
                                                              (eng, slot, eng.gen[slot], node.nid), node.depth))
            elif node.kind == LEAF and lp.diag(slot)["pres"] <= self.retry_res:
                self.retry.append(_Node(bound, node.idx, node.val, RETRY, (eng, slot, eng.gen[slot], node.nid),
                                        node.depth))
            else:
                res.unresolved += 1
                self.unresolved_bounds.append(bound)
            if slot not in self.keep:
                eng.free.append(slot)
            return inc
        if bound >= inc - self._gap_abs(inc):
            eng.free.append(slot)
            return inc
        res.nodes += 1
        if pre is not None:
            flow, z = pre
        else:
            flow = lp.flows([slot])[0]
            z, _ = lp.solution(slot, dense_x=False)
        me = (eng, slot, eng.gen[slot], node.nid)
        for leaf in self._round_all(node, flow, z[self.c0:self.c1]):
            if leaf is not None:
                key = np.packbits(leaf[1] > 0.5).tobytes()
                if key not in self.seen_leaves:
                    self.seen_leaves.add(key)
                    lb = max(bound, self._ibound(*leaf))
                    if lb < inc - self._gap_abs(inc):
                        self.pending.append(_Node(lb, leaf[0], leaf[1], LEAF, me, node.depth + 1))
        if self.primal is not None and (node.depth == 0 or (self.primal_every and res.nodes % self.primal_every == 0)):
            t = time.time()
            for item in self.primal(node.idx, node.val, z, flow):
                idx, val = item[0], item[1]
                sol = item[2] if len(item) > 2 else None
                if sol is not None and sol["objective"] < inc - self._gap_abs(inc):
                    inc = self._heuristic_incumbent(sol)
                key = np.packbits(np.asarray(val) > 0.5).tobytes()
                if key not in self.seen_leaves:
                    self.seen_leaves.add(key)
                    lb = max(bound, self._ibound(idx, val))
                    if lb < inc - self._gap_abs(inc):
                        self.pending.appendleft(_Node(lb, np.asarray(idx), np.asarray(val, np.float64), LEAF, me,
                                                      node.depth + 1))
            res.timing["primal"] += time.time() - t
        var = self._branch_var(node, flow, slot, lp)
        if var is not None:
            for v in (1.0, 0.0):
                idx = np.append(node.idx, var)
                val = np.append(node.val, v)
                cb = max(bound, self._ibound(idx, val))
                if cb >= inc - self._gap_abs(inc):
                    continue
                kind = LEAF if len(idx) >= self._nb else NODE
                heapq.heappush(self.heap, (cb, -(node.depth + 1), next(self.seq),
                                           _Node(cb, idx, val, kind, me, node.depth + 1)))
        eng.free.append(slot)        # most recently finished last: its state survives longest
        return inc

    def _copy_cross(self, cross):
        """Routing warm starts of leaves from their branching nodes' slots of the bound model."""
        for dst, src in cross:
            self.L.lp.copy_routing_from(self.B.lp, src, dst)
            self.res.routing_warm += 1

    def _heuristic_incumbent(self, sol):
        """A checked heuristic point as the incumbent: objective, z and routing (engine rows) taken as given,
        no LP slot behind it (an LP incumbent found later replaces it as usual)."""
        res = self.res
        res.objective = float(sol["objective"])
        res.z = np.asarray(sol["z"], np.float64)
        res.x = self.lp.routing_from_entries(sol["row"], sol["dst"], sol["val"])
        if res.incumbent_slot is not None and res.incumbent_slot in self.keep:
            # (warm=False keeps the LP incumbent in its own working slot: give it back)
            self.keep.discard(res.incumbent_slot)
            self.L.free.append(res.incumbent_slot)
        res.incumbent_slot = None
        res.heuristic_incumbents += 1
        self.inc_node = None
        for e in self.engines:
            e.lp.set_params(self.tol, min(res.objective, self.ub0))
        self.log(f"incumbent {res.objective:.10g} (capacity greedy; lps {res.lps}, nodes {res.nodes})")
        return res.objective

    def _prefetch(self, eng, r, inc):
        """The flows and integer vectors of every branching node in an advance result that will branch (not
        pruned, not infeasible / cut off), read in one device call each: {slot: (flow [F, N], z)}."""
        want = []
        for i, slot in enumerate(r["slots"].tolist()):
            node = self.inflight.get((eng.name, slot))
            st = int(r["status"][i])
            if node is None or node.kind != NODE or st in (LP_INFEASIBLE, LP_CUTOFF):
                continue
            if max(node.bound, float(r["obj"][i])) >= inc - self._gap_abs(inc):
                continue
            want.append(slot)
        if not want:
            return {}
        fl = eng.lp.flows(want)
        zs = eng.lp.solutions(want)
        return {s: (fl[k], zs[k]) for k, s in enumerate(want)}

    def _frontier_hash(self):
        """crc32 of the (sorted) open frontier: bounds, depths, fixings — identical on every rank at the split."""
        import zlib
        h = 0
        for b, d, _, node in self.heap:
            h = zlib.crc32(np.asarray([b, d], np.float64).tobytes(), h)
            h = zlib.crc32(np.asarray(node.idx, np.int64).tobytes(), h)
            h = zlib.crc32(np.asarray(node.val, np.float64).tobytes(), h)
        return int(h)

    def _rebalance(self, inc):
        """Open-node rebalance of the sharded search (one all-gather of the frontier sizes, then one broadcast
        per transfer): every rank whose frontier is empty takes half of the fullest remaining donor's (its
        best-bound nodes, at most `batch`), so a rank whose subtrees died early does not idle.  The pairing
        is computed identically on every rank from the gathered sizes; a moved node starts from its new
        rank's root state."""
        comm = self.comm
        cnt = comm.gather([float(len(self.heap))])[:, 0].astype(np.int64)
        idle = [r for r in range(comm.world) if cnt[r] == 0]
        for r in idle:
            d = int(np.argmax(cnt))
            k = int(min(cnt[d] // 2, self.batch))
            if k <= 0:
                break
            cnt[d] -= k
            cnt[r] += k
            if comm.rank == d:
                give = [heapq.heappop(self.heap)[3] for _ in range(k)]
                head = np.array([k] + [len(n.idx) for n in give], np.float64)
            else:
                head = np.zeros(k + 1)
            head = comm.bcast(head, d)
            lens = head[1:].astype(np.int64)
            tot = int(lens.sum())
            if comm.rank == d:
                meta = np.array([[n.bound, n.depth, n.kind] for n in give], np.float64).ravel()
                body = np.concatenate([meta, np.concatenate([n.idx for n in give]).astype(np.float64) if tot else [],
                                       np.concatenate([n.val for n in give]) if tot else []])
            else:
                body = np.zeros(3 * k + 2 * tot)
            body = comm.bcast(body, d)
            if comm.rank == r:
                meta, idx, val = body[:3 * k].reshape(k, 3), body[3 * k:3 * k + tot], body[3 * k + tot:]
                o = 0
                for q in range(k):
                    n = int(lens[q])
                    node = _Node(float(meta[q, 0]), idx[o:o + n].astype(np.int64), val[o:o + n].copy(),
                                 int(meta[q, 2]), None, int(meta[q, 1]))
                    o += n
                    if node.bound < inc - self._gap_abs(inc):
                        heapq.heappush(self.heap, (node.bound, -node.depth, next(self.seq), node))
                        self.res.rebalanced += 1

    def _trace_entry(self, eng, node, src, budget, bres, cutoff):
        """One submitted node LP for the replay fixture (bench.py's B&B node stream): the node's box (branching
        nodes: their fixings; leaves: the open c / n — every other c and n is fixed to 0), the parent whose
        state warm-started it (None: the model's root state or cold), its model, iteration budget, stops
        (bound_res, gap_tol) and the incumbent cutoff it ran under (None: none yet)."""
        e = {"id": node.nid, "kind": _KIND_NAME[node.kind], "model": eng.name, "depth": node.depth,
             "parent": None if node.parent is None else int(node.parent[3]),
             "warm_from_parent": bool(src is not None and node.parent is not None and src == node.parent[1]),
             "budget": int(budget), "bound_res": float(bres),
             "gap_tol": float(self.bound_gap if (self.two and eng is self.B) else 0.0),
             "cutoff": float(cutoff) if math.isfinite(cutoff) else None}
        if node.kind in (LEAF, RETRY):
            e["open"] = [int(i) for i, v in zip(node.idx, node.val) if v > 0.5]
        else:
            e["fix"] = [[int(i) for i in node.idx], [float(v) for v in node.val]]
        return e

    def _polish(self, res):
        """Re-solve the incumbent leaf from its own final state at polish_tol; keep the result when
        it certifies (the value moves by at most the certificate tolerance)."""
        lp, slot, node = self.lp, res.incumbent_slot, self.inc_node
        lb = np.full((1, lp.n_int), -np.inf)
        ub = np.full((1, lp.n_int), np.inf)
        lb[0, node.idx] = node.val
        ub[0, node.idx] = node.val
        st = lp.submit(np.array([slot], np.int32), lb, ub, tol=self.polish_tol, cutoff=math.inf,
                       max_iters=self.polish_iters, check_every=self.check_every, warm_start=True)
        if int(st[0]) == LP_INFEASIBLE:
            return
        r = lp.advance(1)
        while lp.active() > 0:
            r = lp.advance(1)
        if len(r["slots"]) and int(r["status"][0]) == LP_OPTIMAL:
            res.objective = float(r["primal_obj"][0])
            res.z, _ = lp.solution(slot, dense_x=False)
            res.x = lp.routing(slot)
            res.polished = True
        # (uncertified: the slot's state moved on; res.x / res.z stay the certified leaf's, fetched before)

    def _finish_sharded(self, res, inc, limit_hit, unresolved_below, any_unresolved=None):
        """End of a sharded search: one all-gather of every rank's summary; the owner of the best
        certified incumbent (lowest rank on ties, chosen on the certified objectives BEFORE any polish)
        polishes it and broadcasts objective, integer vector and compacted routing entries."""
        comm, lp = self.comm, self.lp
        mine = res.objective is not None and res.objective <= inc
        g = comm.gather([res.bound, 1.0 if limit_hit else 0.0, 1.0 if unresolved_below else 0.0, 1.0 if mine else 0.0,
                         res.nodes - self.presplit[0], res.lps - self.presplit[1], res.certified - self.presplit[2],
                         1.0 if (any_unresolved if any_unresolved is not None else self.unresolved_bounds) else 0.0])
        res.bound = float(g[:, 0].min())
        self._limit_hit = bool(g[:, 1].max() > 0)
        self._unresolved_below = bool(g[:, 2].max() > 0)
        self._any_unresolved = bool(g[:, 7].max() > 0)
        # the pre-split phase ran identically on every rank: count it once
        res.nodes = int(g[:, 4].sum()) + self.presplit[0]
        res.lps = int(g[:, 5].sum()) + self.presplit[1]
        res.certified = int(g[:, 6].sum()) + self.presplit[2]
        owners = np.flatnonzero(g[:, 3] > 0)
        if owners.size == 0:
            res.objective, res.z, res.x = None, None, None
            return
        owner = int(owners[0])
        own = comm.rank == owner
        if own:
            if res.incumbent_slot is not None:      # (a heuristic incumbent carries its routing already)
                res.x = lp.routing(res.incumbent_slot)
                if self.polish_tol:
                    self._polish(res)
            head = np.array([res.objective, 1.0 if res.polished else 0.0, float(len(res.x.row))])
        else:
            head = np.zeros(3)
        head = comm.bcast(head, owner)
        k = int(head[2])
        z = comm.bcast(np.asarray(res.z if own else np.zeros(lp.n_int), np.float64), owner)
        row = comm.bcast(np.asarray(res.x.row if own else np.zeros(k), np.int32), owner)
        dst = comm.bcast(np.asarray(res.x.dst if own else np.zeros(k), np.int32), owner)
        val = comm.bcast(np.asarray(res.x.val if own else np.zeros(k), np.float64), owner)
        res.objective, res.polished, res.z = float(head[0]), bool(head[1] > 0), z
        res.x = lp.routing_from_entries(row, dst, val)

    # ---------------------------------------------------------------------------------------
    def _native_ok(self, comm):
        """The native tree runs every search without per-node Python callbacks — single rank or sharded (API 12) —
        on the engine's models by default, and on any Python model with the streaming interface (the CPU suite's
        HiGHS node LPs, through lp.PyBnbEngine) when native=True."""
        if self.native is False or os.environ.get("NEP_BNB_PYTHON", "0") not in ("", "0"):
            return False
        s2 = self.step2_native is not None and os.environ.get("NEP_BNB_STEP2", STEP2_NATIVE_DEFAULT) not in ("", "0")
        engine = hasattr(self.lp, "_h") and (self.bound_lp is None or hasattr(self.bound_lp, "_h"))
        eligible = (self.trace is None and (self.integer_bound is None or s2) and (self.improve is None or s2)
                    and (self.branching == 0 or self.native is not False)
                    and not self.leaf_routing_warm and self.primal_every == 0 and (engine or self.native is True))
        if comm.world > 1 and os.environ.get("NEP_BNB_SHARDED_NATIVE", "1") in ("", "0"):
            eligible = False
        if self.native and not eligible:
            raise ValueError("native tree search: no trace / leaf routing warm starts / primal_every, "
                             "integer_bound and improve only with step2_native")
        return eligible

    def _rebalance_native(self, lib, tree, heap_n):
        """_rebalance on the native tree: the same pairing from one all-gather of the heap sizes, the donor's k
        best-bound open nodes exported (nep_bnb_export_nodes) and broadcast, imported by the idle rank (pruned
        against the agreed incumbent; they start from that rank's root state)."""
        from .lp import _check, _ptr
        comm = self.comm
        cnt = comm.gather([float(heap_n)])[:, 0].astype(np.int64)
        idle = [r for r in range(comm.world) if cnt[r] == 0]
        nb = self._nb + 1
        for r in idle:
            d = int(np.argmax(cnt))
            k = int(min(cnt[d] // 2, self.batch))
            if k <= 0:
                break
            cnt[d] -= k
            cnt[r] += k
            if comm.rank == d:
                lens = np.zeros(k, np.int32)
                meta = np.zeros(3 * k)
                idx = np.zeros(k * nb, np.int32)
                val = np.zeros(k * nb)
                _check(lib, lib.nep_bnb_export_nodes(tree, k, k * nb, _ptr(lens), _ptr(meta), _ptr(idx), _ptr(val)),
                       "nep_bnb_export_nodes")
                tot = int(lens.sum())
                head = np.concatenate([[k], lens.astype(np.float64)])
            else:
                head = np.zeros(k + 1)
            head = comm.bcast(head, d)
            lens = head[1:].astype(np.int32)
            tot = int(lens.sum())
            if comm.rank == d:
                body = np.concatenate([meta, idx[:tot].astype(np.float64), val[:tot]])
            else:
                body = np.zeros(3 * k + 2 * tot)
            body = comm.bcast(body, d)
            if comm.rank == r:
                meta = np.ascontiguousarray(body[:3 * k])
                idx = np.ascontiguousarray(body[3 * k:3 * k + tot].astype(np.int32))
                val = np.ascontiguousarray(body[3 * k + tot:])
                _check(lib, lib.nep_bnb_import_nodes(tree, k, _ptr(lens), _ptr(meta), _ptr(idx), _ptr(val)),
                       "nep_bnb_import_nodes")

    def _solve_native(self):
        """solve() on the native tree (nep_bnb_*, csrc/nep_bnb.cpp): the same search, its loop in the library;
        this method handles the root's primal heuristic (NEP_BNB_ROOT) and the end (routing, polish, repair)."""
        import ctypes
        from .lp import BnbParams, BnbStats, PyBnbEngine, _check, _ptr, load_library
        t0 = self.t0 = time.time()
        self.res = res = BnBResult()
        comm = self.comm
        lp = self.lp
        lib = getattr(lp, "_lib", None) or load_library()
        n0, n1 = self.n_range if self.n_range is not None else (-1, -1)
        inf = math.inf
        p = BnbParams(c0=self.c0, c1=self.c1, n0=n0, n1=n1, n_int=lp.n_int, F=self.F, N=self.N,
                      warm=1 if self.warm else 0, batch=int(self.batch), batch_b=int(self.batch_b),
                      check_every=int(self.check_every),
                      root_check_every=int(self.root_check_every), unit_flow_leaves=1 if len(self.round_modes) > 2 else 0,
                      objective_integral=1 if self.objective_integral else 0,
                      primal_at_root=1 if self.primal is not None else 0, tol=self.tol, gap=self.gap,
                      bound_gap=self.bound_gap, max_iters=int(self.max_iters), node_max_iters=int(self.node_max_iters),
                      root_max_iters=int(self.root_max_iters), node_bound_res=float(self.node_bound_res or 0.0),
                      retry_res=float(self.retry_res), flow_tol=float(self.flow_tol), upper_bound=float(self.ub0),
                      # (round-5 ADVICE: a non-finite node limit is no limit)
                      node_limit=int(min(float(self.node_limit), 2.0 ** 62)), time_limit=float(self.time_limit or 0.0),
                      world=int(comm.world), rank=int(comm.rank), branching=self.branching,
                      strong_cands=self.strong_cands, strong_rel=self.strong_rel, strong_iters=self.strong_iters,
                      objective_unit=float(self.objective_unit))
        py_engines = []
        if hasattr(lp, "_h"):
            tree = lib.nep_bnb_create(lp._h, self.bound_lp._h if self.two else None, ctypes.byref(p),
                                      _ptr(self.fn_mem), _ptr(self.node_mem))
        else:
            py_engines = [PyBnbEngine(lp, self.F, self.N)] + ([PyBnbEngine(self.bound_lp, self.F, self.N)]
                                                              if self.two else [])
            tree = lib.nep_bnb_create_engines(ctypes.byref(py_engines[0].table),
                                              ctypes.byref(py_engines[1].table) if self.two else None,
                                              ctypes.byref(p), _ptr(self.fn_mem), _ptr(self.node_mem))
        if not tree:
            raise RuntimeError(f"nep_bnb_create failed: {lib.nep_last_error().decode()}")

        def run_checked(what, rc):
            for e in py_engines:
                if e.error is not None:
                    raise e.error
            _check(lib, rc, what)

        bm = self.bound_lp if self.two else lp
        loops = 0
        split_seen = False
        try:
            if self.step2_native is not None:
                create, cap, old = self.step2_native
                old = np.ascontiguousarray(old, np.float64).reshape(-1)
                _check(lib, lib.nep_bnb_set_step2(tree, 1 if create else 0, float(cap), _ptr(old),
                                                  1 if self.improve is not None else 0), "nep_bnb_set_step2")
            for idx, val in self.seed_leaves:
                idx = np.ascontiguousarray(idx, np.int32)
                val = np.ascontiguousarray(val, np.float64)
                _check(lib, lib.nep_bnb_add_leaf(tree, len(idx), _ptr(idx), _ptr(val), -inf, 0), "nep_bnb_add_leaf")
            ev = ctypes.c_int32()
            sync = np.zeros(6)
            while True:
                run_checked("nep_bnb_run", lib.nep_bnb_run(tree, ctypes.byref(ev)))
                if ev.value == 0:
                    break
                if ev.value == 3:
                    # NEP_BNB_SYNC (sharded): the loop's one collective — incumbent MIN, stop OR, open SUM — then,
                    # every rebalance_every loops after the split, the open-node rebalance
                    _check(lib, lib.nep_bnb_sync_get(tree, _ptr(sync)), "nep_bnb_sync_get")
                    inc_l, stop_l, open_l, heap_n, split = float(sync[0]), bool(sync[1]), int(sync[2]), int(sync[3]), \
                        bool(sync[4])
                    inc_g, stop_g, total = comm.agree(inc_l, stop_l, open_l)
                    _check(lib, lib.nep_bnb_sync_set(tree, inc_g, 1 if stop_g else 0, int(total)), "nep_bnb_sync_set")
                    split_seen = split_seen or split
                    if not stop_g and (total if split else open_l) > 0:
                        loops += 1
                        if split and self.rebalance_every and loops % self.rebalance_every == 0:
                            self._rebalance_native(lib, tree, heap_n)
                    continue
                if ev.value == 2:
                    # NEP_BNB_INCUMBENT: the neighbour leaves of a new LP incumbent (step 2's node relocation)
                    n_fix = ctypes.c_int32()
                    idx = np.zeros(self._nb + 1, np.int32)
                    val = np.zeros(self._nb + 1)
                    value = ctypes.c_double()
                    _check(lib, lib.nep_bnb_incumbent_event(tree, ctypes.byref(n_fix), _ptr(idx), _ptr(val),
                                                            ctypes.byref(value)), "nep_bnb_incumbent_event")
                    k = n_fix.value
                    self.log(f"incumbent {value.value:.10g}")
                    for nidx, nval in self.improve(idx[:k].astype(np.int64), val[:k].copy(), value.value):
                        nidx = np.ascontiguousarray(nidx, np.int32)
                        nval = np.ascontiguousarray(nval, np.float64)
                        _check(lib, lib.nep_bnb_add_leaf(tree, len(nidx), _ptr(nidx), _ptr(nval), -inf, 2),
                               "nep_bnb_add_leaf")
                    continue
                # NEP_BNB_ROOT: the primal heuristic on the root branching node's LP
                t = time.time()
                z = np.zeros(bm.n_int)
                flow = np.zeros((self.F, self.N), np.float32)
                _check(lib, lib.nep_bnb_event_data(tree, _ptr(z), _ptr(flow)), "nep_bnb_event_data")
                inc = res.objective if res.objective is not None else inf
                for item in self.primal(np.zeros(0, np.int64), np.zeros(0), z, flow):
                    idx, val = np.ascontiguousarray(item[0], np.int32), np.ascontiguousarray(item[1], np.float64)
                    sol = item[2] if len(item) > 2 else None
                    if sol is not None and sol["objective"] < inc - self._gap_abs(inc):
                        res.objective = inc = float(sol["objective"])
                        res.z = np.asarray(sol["z"], np.float64)
                        res.x = self.lp.routing_from_entries(sol["row"], sol["dst"], sol["val"])
                        _check(lib, lib.nep_bnb_set_incumbent(tree, inc), "nep_bnb_set_incumbent")
                        self.log(f"incumbent {inc:.10g} (capacity greedy)")
                    _check(lib, lib.nep_bnb_add_leaf(tree, len(idx), _ptr(idx), _ptr(val), -inf, 1), "nep_bnb_add_leaf")
                res.timing["primal"] += time.time() - t
            st = BnbStats()
            _check(lib, lib.nep_bnb_get_stats(tree, ctypes.byref(st)), "nep_bnb_get_stats")
            its = np.zeros(max(1, st.n_lp_iters), np.int64)
            _check(lib, lib.nep_bnb_get_lp_iters(tree, _ptr(its)), "nep_bnb_get_lp_iters")
            res.lp_iters = its[:st.n_lp_iters].tolist()
            if st.incumbent_source == 1:
                n_fix = ctypes.c_int32()
                z = np.zeros(lp.n_int)
                idx = np.zeros(self._nb + 1, np.int32)
                val = np.zeros(self._nb + 1)
                _check(lib, lib.nep_bnb_incumbent(tree, _ptr(z), ctypes.byref(n_fix), _ptr(idx), _ptr(val)),
                       "nep_bnb_incumbent")
                res.objective, res.z = float(st.incumbent), z
                res.incumbent_slot = int(st.incumbent_slot)
                k = n_fix.value
                self.inc_node = _Node(st.incumbent, idx[:k].astype(np.int64), val[:k].copy(), LEAF, None, 0)
            elif st.incumbent_source == 0:
                res.objective = None
        finally:
            lib.nep_bnb_destroy(tree)
        names = ("certified", "bound", "limit", "infeasible", "cutoff", "numerical", "presolve_infeasible")
        res.lp_status = {k: int(st.lp_status[i]) for i, k in enumerate(names)}
        res.lp_status_kind = {kn: {k: int(st.lp_status_kind[q][i]) for i, k in enumerate(names)}
                              for q, kn in ((NODE, "node"), (LEAF, "leaf"), (RETRY, "retry"), (REFROOT, "refroot"))}
        for k in ("nodes", "leaves", "lps", "certified", "lp_iterations", "unresolved", "drained", "advance_calls",
                  "inflight_sum", "heuristic_incumbents"):
            setattr(res, k, int(getattr(st, k)))
        res.heuristic_incumbents = int(st.heuristic_incumbents)
        tm = res.timing
        tm["advance"], tm["finish"], tm["submit"] = st.advance_seconds, st.finish_seconds, st.submit_seconds
        tm["drain"], tm["root"] = st.drain_seconds, st.root_seconds
        res.native = True
        res.rebalanced = int(st.rebalanced)
        res.strong = {k: int(getattr(st, k)) for k in ("strong_nodes", "strong_lps", "strong_iterations",
                                                       "strong_decided")}
        res.split_hash = int(st.split_hash) if split_seen else None
        t_end = time.perf_counter()
        res.bound = float(st.bound)
        limit_hit, unresolved_below = bool(st.limit_hit), bool(st.unresolved_below)
        if comm.world == 1:
            if res.objective is not None and res.incumbent_slot is not None:
                res.x = lp.routing(res.incumbent_slot)
                if self.polish_tol:
                    self._polish(res)
        else:
            self.presplit = (int(st.presplit_nodes), int(st.presplit_lps), int(st.presplit_certified)) \
                if split_seen else (res.nodes, res.lps, res.certified)
            self._finish_sharded(res, float(st.agreed_incumbent), limit_hit, unresolved_below,
                                 any_unresolved=bool(st.any_unresolved))
            limit_hit, unresolved_below = self._limit_hit, self._unresolved_below
        if res.objective is not None and self.repair is not None:
            res.x, dobj, res.repaired = self.repair(res.x, res.z)
            res.objective += dobj
            if not res.repaired:
                self.log("incumbent routing: CPU repair incomplete")
        any_unresolved = bool(st.any_unresolved) if comm.world == 1 else self._any_unresolved
        if res.objective is None:
            res.status = LIMIT if (limit_hit or any_unresolved) else INFEASIBLE
        else:
            res.status = LIMIT if (limit_hit or unresolved_below) else OPTIMAL
        if st.stalled:
            self.log("search stalled: open nodes could not get an LP slot (reported as a limit)")
        res.timing["end"] = time.perf_counter() - t_end
        res.seconds = time.time() - t0
        return res

    def solve(self):
        if self._native_ok(self.comm):
            return self._solve_native()
        t0 = self.t0 = time.time()
        self.res = res = BnBResult()
        lp = self.lp
        comm = self.comm
        inc = math.inf
        self.seq = itertools.count()
        rb = self._ibound(np.zeros(0, np.int64), np.zeros(0))
        root = _Node(rb, np.zeros(0, np.int64), np.zeros(0), NODE, None, 0)
        self.heap = [] if rb == math.inf else [(rb, 0, next(self.seq), root)]
        self.pending = deque()       # rounding leaves
        self.retry = deque()         # uncertified leaves, re-solved once with the root budget
        self.unresolved_bounds = []
        self.seen_leaves = set()
        self.inflight = {}           # (engine name, slot) -> node
        self.keep = set()
        self.inc_node = None
        self.nid_seq = itertools.count()
        L = _Engine(lp, self.reserved, "leaf")
        B = L if not self.two else _Engine(self.bound_lp, 1 if self.warm else 0, "bound")
        self.L, self.B = L, B
        self.engines = [L] if not self.two else [B, L]
        # two models: the reference root LP (the leaves' warm-start state) runs beside the first bound LPs
        self.refroot = None
        if self.two:
            if self.warm:
                self.refroot = _Node(-math.inf, np.zeros(0, np.int64), np.zeros(0), REFROOT, None, 0)
            else:
                L.root_ready = True
        sharded = comm.world == 1
        self.presplit = (0, 0, 0)
        limit_hit = False
        while True:
            if not sharded and len(self.heap) >= comm.world * self.batch and not self.inflight:
                # deal the (identical on every rank) frontier: canonical order, round robin
                self.heap.sort(key=lambda h: h[:3])
                res.split_hash = self._frontier_hash()
                self.heap = [h for i, h in enumerate(self.heap) if i % comm.world == comm.rank]
                heapq.heapify(self.heap)
                self.pending = deque(lf for i, lf in enumerate(self.pending) if i % comm.world == comm.rank)
                self.retry = deque(lf for i, lf in enumerate(self.retry) if i % comm.world == comm.rank)
                self.presplit = (res.nodes, res.lps, res.certified)
                sharded = True
            stop = res.nodes >= self.node_limit or bool(self.time_limit and time.time() - t0 > self.time_limit)
            busy = sum(1 for n in self.inflight.values() if n.kind != REFROOT)
            open_n = len(self.heap) + len(self.pending) + len(self.retry) + busy
            if comm.world > 1:
                # every rank takes the same stop / termination decision in the same loop iteration: one
                # collective carries the incumbent (MIN), the stop flags (OR) and the open counts (SUM)
                inc, stop, total = comm.agree(inc, stop, open_n)
                open_n = total if sharded else open_n
            if open_n == 0:
                break
            if stop:
                limit_hit = True
                break
            loops = getattr(self, "_loops", 0) + 1
            self._loops = loops
            if sharded and comm.world > 1 and self.rebalance_every and loops % self.rebalance_every == 0:
                self._rebalance(inc)
            # fill the free slots: retries, rounding leaves, then best-first open nodes
            items = []
            # at most `batch` LPs in flight per model; slots beyond that keep finished states (parked
            # parents, least recently finished reused first)
            capL = self.batch - L.inflight
            capB = self.batch_b - B.inflight
            if not self.two:
                while L.free and capL > 0 and (self.retry or self.pending or self.heap):
                    if self.retry:
                        node = self.retry.popleft()
                    elif self.pending:
                        node = self.pending.popleft()
                        if node.bound >= inc - self._gap_abs(inc):
                            continue
                    else:
                        _, _, _, node = heapq.heappop(self.heap)
                        if node.bound >= inc - self._gap_abs(inc):
                            continue
                    items.append((L, L.free.popleft(), node))
                    capL -= 1
                    if not L.root_ready:
                        break                 # the root runs alone (its state warm-starts everything after)
            else:
                if self.refroot is not None and L.free and capL > 0:
                    items.append((L, L.free.popleft(), self.refroot))
                    capL -= 1
                    self.refroot = None
                # (the branching nodes wait for both roots: 32 bound LPs beside the lone reference root would
                # starve its one-slot blocks — 512x256: not done after 60 s, 1.8 s alone)
                while B.free and capB > 0 and self.heap and (not B.root_ready or L.root_ready):
                    _, _, _, node = heapq.heappop(self.heap)
                    if node.bound >= inc - self._gap_abs(inc):
                        continue
                    if node.kind != NODE:          # a leaf from branching: the reference model's
                        self.pending.append(node)
                        continue
                    items.append((B, B.free.popleft(), node))
                    capB -= 1
                    if not B.root_ready:
                        break
                while L.root_ready and L.free and capL > 0 and (self.retry or self.pending):
                    node = self.retry.popleft() if self.retry else self.pending.popleft()
                    if node.kind == LEAF and node.bound >= inc - self._gap_abs(inc):
                        continue
                    items.append((L, L.free.popleft(), node))
                    capL -= 1
            tm = res.timing
            t1 = time.perf_counter()
            if items:
                self._submit(items, inc)
            t2 = time.perf_counter()
            tm["submit"] += t2 - t1
            if not self.inflight:
                continue
            # before the frontier is dealt every rank must stay identical: drain each batch whole.  Under a
            # time limit the sharded loop comes back after every block, so a stop is never held up by
            # long LPs (a leaf's retry runs the root budget).  Two models: one block of each per loop (each
            # pipelines its next block before returning, so both streams keep iterating)
            res.advance_calls += 1
            res.inflight_sum += busy
            for eng in self.engines:
                if eng.inflight <= 0:
                    continue
                if self.two:
                    r = eng.lp.advance(0 if sharded else eng.inflight)
                else:
                    r = eng.lp.advance((0 if self.time_limit else 1) if sharded else eng.inflight)
                t3 = time.perf_counter()
                tm["advance"] += t3 - t2
                fl = self._prefetch(eng, r, inc)
                for i, slot in enumerate(r["slots"].tolist()):
                    node = self.inflight.pop((eng.name, slot))
                    inc = self._finish(eng, slot, node, int(r["status"][i]), float(r["obj"][i]),
                                       float(r["primal_obj"][i]), int(r["iters"][i]), inc, fl.get(slot))
                t2 = time.perf_counter()
                tm["finish"] += t2 - t3
        # drain what still iterates (a stop decision): a cutoff of -inf stops every LP in flight at its next
        # certificate check (one block), with its best Lagrangian bound, which stays valid for its node
        t_end = time.perf_counter()
        open_bounds = [n.bound for n in self.inflight.values() if n.kind != REFROOT]
        res.drained = len(open_bounds)
        for eng in self.engines:
            if eng.lp.active() > 0:
                eng.lp.set_params(self.tol, -math.inf)
        for eng in self.engines:
            while eng.lp.active() > 0:
                r = eng.lp.advance(eng.lp.active())
                for i, slot in enumerate(r["slots"].tolist()):
                    node = self.inflight.pop((eng.name, slot), None)
                    if node is not None and node.kind != REFROOT and int(r["status"][i]) != LP_INFEASIBLE:
                        open_bounds.append(max(node.bound, float(r["obj"][i])))
        res.timing["drain"] = time.perf_counter() - t_end
        t_end = time.perf_counter()
        open_bounds += [h[0] for h in self.heap] + [n.bound for n in self.pending] + [n.bound for n in self.retry]
        open_bounds += self.unresolved_bounds
        res.bound = min(open_bounds + [inc])
        unresolved_below = any(b < inc - self._gap_abs(inc) for b in self.unresolved_bounds)
        if comm.world == 1:
            if res.objective is not None and res.incumbent_slot is not None:
                # the certified leaf's routing, fetched once (compacted on the device) before the
                # polish re-solve may move the slot
                res.x = lp.routing(res.incumbent_slot)
                if self.polish_tol:
                    self._polish(res)
        else:
            self._finish_sharded(res, inc, limit_hit, unresolved_below)
            limit_hit, unresolved_below = self._limit_hit, self._unresolved_below
        if res.objective is not None and self.repair is not None:
            # identical on every rank (the owner's routing was broadcast)
            res.x, dobj, res.repaired = self.repair(res.x, res.z)
            res.objective += dobj
            if not res.repaired:
                self.log("incumbent routing: CPU repair incomplete")
        any_unresolved = bool(self.unresolved_bounds) if comm.world == 1 else self._any_unresolved
        if res.objective is None:
            res.status = LIMIT if (limit_hit or any_unresolved) else INFEASIBLE
        else:
            res.status = LIMIT if (limit_hit or unresolved_below) else OPTIMAL
        res.timing["end"] = time.perf_counter() - t_end
        res.seconds = time.time() - t0
        return res
