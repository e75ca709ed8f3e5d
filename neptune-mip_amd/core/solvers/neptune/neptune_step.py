"""NEPTUNE step models on the MI355X engine.

Reference classes (same names, constructor keywords and side effects on `Data`):
  NeptuneStepBase / NeptuneStep1CPU*     `core/solvers/neptune/neptune_step1.py:5-77`
  NeptuneStep2Base / NeptuneStep2*       `core/solvers/neptune/neptune_step2.py:5-93`
The reference enumerates the model row by row through pywraplp (`neptune/utils/variables.py`,
`constraints_step1.py`, `constraints_step2.py`, `objectives.py`) and hands it to SCIP.  Here the
same model is built structurally by the engine (`nep_model_create`, csrc/nep_host.cpp build(); row
map in DESIGN.md §2) and solved by the batched GPU branch-and-bound (core/engine/bnb.py).

results() returns x[i][f][j] and c[f][j] of the reference's `output_x_and_c`
(`neptune/utils/output.py:5-15`): c dense, x as a core.engine.routing.SparseRouting (the
device-compacted nonzeros; `np.asarray(x)` gives the dense matrix on demand, the wire format is built
from the entries); step 1 stores them in data.prev_x / prev_c (`neptune_step1.py:21-27`) and the
utilisation variants data.prev_n (:55-60).
"""
import math

import numpy as np

from ...engine import lp as _lp
from ...engine.bnb import OPTIMAL, BranchAndBound
from ...engine.heuristics import capacity_greedy
from ...engine.routing import SparseRouting, repair_cpu
from ..solver import Solver


def make_lp(data, variant, step, max_batch, **kw):
    """The engine model of one step (indirection kept so tests can substitute the CPU oracle)."""
    return _lp.LPModel(data, variant, step=step, max_batch=max_batch, **kw)


class NeptuneStepBase(Solver):
    VARIANT = None

    def __init__(self, batch=16, node_limit=20000, time_limit=None, lp_tol=5e-7, lp_max_iters=5000, **kwargs):
        super().__init__(**kwargs)
        self.batch = batch
        self.node_limit = node_limit
        self.time_limit = time_limit
        self.lp_tol = lp_tol
        # node-LP iteration limit of the B&B (the bound of a stopped LP stays valid).  Measured on the
        # golden flows: 5000 instead of 100000 gives the same scores 13-18x faster (payload.json
        # 28.0 s -> 1.5 s): step-2 LPs that do not certify stop early
        self.lp_max_iters = lp_max_iters
        self.result = None
        self.x_matrix = None
        self.c_matrix = None
        self.n_vector = None

    # the model is structured: nothing to enumerate (reference variables.py / constraints_*.py)
    def init_vars(self):
        pass

    def init_constraints(self):
        pass

    def init_objective(self):
        pass

    def step_id(self):
        return _lp.STEP1

    def model_kwargs(self):
        return {}

    def upper_bound(self):
        return math.inf

    # B&B branching nodes stop once their bound has converged (core/engine/bnb.py, NEP_LP_BOUND); step 2
    # keeps every node LP to its certificate: its disruption objective (weights F N) moves by orders of
    # magnitude with the residual, so a node stopped at 1e-2 can branch on flows far from its LP optimum
    node_bound_res = 1e-2
    # the unit-flow rounding leaf (core/engine/bnb.py): step 1 only — on step 2 it mostly adds leaves whose
    # placement leaves the routing infeasible, which the node LPs cannot prove, so the search ends LIMIT
    unit_flow_leaves = True
    # step-1 branching nodes stop at a quarter of the leaves' node-LP limit (their bound is valid wherever
    # they stop): 256x128 / 20 s: 3678 vs 3274 node LPs, bound 0.00607 vs 0.00596, same incumbent;
    # 512x256 / 45 s: bound 0.00264 vs 0.00243, incumbent 0.5474 vs 0.5483
    node_iters_fraction = 0.25
    # the native tree's branching rule (core/engine/bnb.py): step 1 uses reliability branching — pseudo-costs, strong-
    # branching probe LPs while a candidate's pseudo-costs are unreliable (DESIGN.md §7 "Branching rules": 64x32 bound
    # after 20k nodes 0.13533 against 0.13495 with the flow rule, 48x24 / 56x28 likewise); step 2 keeps the flow rule
    branching = 2

    def seed_leaves(self, layout):
        """Placements to try as leaves right after the root (a B&B primal start); none by default."""
        return []

    # the branching nodes' bounds come from the facility relaxation (NEP_RELAX_FACILITY: x <= c, c <= n in place
    # of the big-M pairs; include/neptune_lp.h) where it exists — step 1 with n (MinUtilization,
    # MinDelayAndUtilization); leaves stay on the reference model
    strengthen = True

    # bound-model slots beyond the `batch` in flight and its root's: finished branching nodes' states stay there
    # (least recently finished reused first) so their children warm-start from them (DESIGN.md §7 "Parked parents")
    bound_park = 0

    def bound_model(self, data, max_batch):
        if not self.strengthen or self.step_id() != _lp.STEP1 or self.VARIANT == "MinDelay":
            return None
        return make_lp(data, self.VARIANT, self.step_id(), max_batch + int(self.bound_park),
                       relaxation=_lp.RELAX_FACILITY, **self.model_kwargs())

    def integer_bound(self, layout=None):
        """bound(idx, val): a lower bound on the objective of every integral completion of a node's
        fixings (+inf: none exists), or None."""
        return None

    def native_bound(self):
        """integer_bound's parameters for the native tree search (nep_bnb_set_step2), or None."""
        return None

    def objective_integral(self):
        """Every integral point of the step model has an integral objective: step-1 MinUtilization (sum n,
        objectives.py:24-27) and every step 2 (minimize_disruption, objectives.py:55-63: integer weights on
        binaries and integers) — True; step-1 MinDelayAndUtilization without workload (objectives.py:34-35 sets no
        x terms when sum W = 0: alpha / N sum n) — its unit alpha / N; else False."""
        if self.step_id() != _lp.STEP1 or self.VARIANT == "MinUtilization":
            return True
        if self.VARIANT == "MinDelayAndUtilization" and not np.asarray(self.data.workload_matrix).any():
            return float(self.alpha) / len(self.data.nodes)
        return False

    def objective_weights(self):
        """(cost per open node, coefficient of sum W D of the routing) of the step-1 objective, or None."""
        return None

    def primal_heuristic(self, layout, row_map=None):
        """primal(idx, val, z, flow) -> [(idx, val, sol)]: capacity-greedy leaves of a branching node (core/engine/
        heuristics.py), the LP's n ranking the nodes; None where the objective has no node count.
        sol (with row_map = the model's (row_f, row_src)): the greedy point itself as an incumbent —
        {"objective", "z", "row", "dst", "val"} — when it passes check_placement in fp64, else None."""
        wts = self.objective_weights()
        if wts is None or layout.get("n") is None:
            return None
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        c0, c1 = layout["c"]
        n0, n1 = layout["n"]
        W = np.asarray(d.workload_matrix, np.float64)
        D = np.asarray(d.node_delay_matrix, np.float64)
        cpr = np.asarray(d.core_per_req_matrix, np.float64)
        cores = np.asarray(d.node_cores_matrix, np.float64).reshape(N)
        fmem = np.asarray(d.function_memory_matrix, np.float64).reshape(F)
        nmem = np.asarray(d.node_memory_matrix, np.float64).reshape(N)

        def primal(idx, val, z, flow):
            idx = np.asarray(idx)
            cfix = np.full(F * N, -1.0)
            sel = (idx >= c0) & (idx < c1)
            cfix[idx[sel] - c0] = np.asarray(val)[sel]
            nfix = np.full(N, -1.0)
            sel = (idx >= n0) & (idx < n1)
            nfix[idx[sel] - n0] = np.asarray(val)[sel]
            out = []
            for C, n, _, route in capacity_greedy(W, D, cpr, cores, fmem, nmem, np.asarray(z[n0:n1], np.float64),
                                                  flow=flow, tries=3, node_cost=wts[0], delay_coef=wts[1],
                                                  new_pen=1.0,
                                                  c_fix=cfix.reshape(F, N), n_fix=nfix):
                sol = None if row_map is None else self._greedy_incumbent(C, n, route, row_map, wts, layout)
                out.append((np.concatenate([np.arange(c0, c1), np.arange(n0, n1)]), np.concatenate([C.ravel(), n]),
                            sol))
            return out
        return primal

    def _greedy_incumbent(self, C, n, route, row_map, wts, layout):
        """The greedy's placement and routing as a feasible point of the reference model, in the engine's
        aggregated rows (every loaded source's row to its node, each pooled zero-workload row to one open
        placement of its function), with its objective computed from the reference's objective
        (objectives.py:13-53) — or None when check_placement rejects it."""
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        W = np.asarray(d.workload_matrix, np.float64)
        D = np.asarray(d.node_delay_matrix, np.float64)
        rf, rs = (np.asarray(a) for a in row_map)
        rowid = {(int(f), int(i)): r for r, (f, i) in enumerate(zip(rf.tolist(), rs.tolist()))}
        f_, i_, j_ = route
        dst = np.full(len(rf), -1, np.int64)
        for f, i, j in zip(f_.tolist(), i_.tolist(), j_.tolist()):
            r = rowid.get((f, i))
            if r is None:
                return None
            dst[r] = j
        for r in np.flatnonzero(dst < 0):
            f = int(rf[r])
            opened = np.flatnonzero(C[f] > 0.5)
            if opened.size == 0:
                return None
            if rs[r] >= 0 and W[f, rs[r]] > 0:
                return None                      # a loaded source the greedy left unrouted
            dst[r] = int(opened[0])
        x_fij = np.zeros((F, N, N))              # x[f, i, j] (the pooled rows expanded over their sources)
        for r in range(len(rf)):
            f, i = int(rf[r]), int(rs[r])
            if i >= 0:
                x_fij[f, i, dst[r]] = 1.0
            else:
                for i0 in np.flatnonzero(W[f] == 0):
                    x_fij[f, i0, dst[r]] = 1.0
        if not self.check_placement(C, n, x_fij):
            return None
        obj = wts[0] * float(n.sum()) + wts[1] * float(np.einsum("fi,ij,fij->", W, D, x_fij))
        c0, c1 = layout["c"]
        n0, n1 = layout["n"]
        z = np.zeros(max(c1, n1))
        z[c0:c1] = C.ravel()
        z[n0:n1] = n
        return {"objective": obj, "z": z, "row": np.arange(len(rf)), "dst": dst, "val": np.ones(len(rf))}

    def check_placement(self, C, n, x):
        """Every step-1 row of the reference (constraints_step1.py) at an integral point, in fp64: C1/C2 (flow
        only into open placements, >= 1 - eps into each), C3 memory, C4 each source routed once, C5 CPU
        (<= cores + 1e-6, the checker's tolerance), C6/C7 (n = any placement), C8 budget."""
        d = self.data
        W = np.asarray(d.workload_matrix, np.float64)
        cpr = np.asarray(d.core_per_req_matrix, np.float64)
        col = x.sum(axis=1)                                                       # [f, j]
        if (col > 1e6 * C + 1e-9).any() or (col < C - 1e-6 - 1e-12).any():
            return False
        if ((np.asarray(d.function_memory_matrix, np.float64) @ C) > np.asarray(d.node_memory_matrix, np.float64) + 1e-9).any():
            return False
        if np.abs(x.sum(axis=2) - 1.0).max() > 1e-12:
            return False
        cpu = np.einsum("fi,fj,fij->j", W, cpr, x)
        if (cpu > np.asarray(d.node_cores_matrix, np.float64) + 1e-6).any():
            return False
        used = C.sum(axis=0)
        if (used > 1e6 * n + 1e-9).any() or (used < n - 1e-6).any():
            return False
        # C8 is one row per node, n[j] * node_costs[j] <= node_budget (constraints_step1.py:101-103), not a sum
        cost = np.asarray(getattr(d, "node_costs", np.zeros(len(n))), np.float64)
        budget = float(getattr(d, "node_budget", np.inf))
        return bool((cost * n <= budget + 1e-9).all())

    def improve(self, layout):
        """improve(idx, val, value) -> [(idx, val)]: neighbour placements of a new incumbent leaf
        worth solving (a local-search heuristic), or None."""
        return None

    def routing_coef(self):
        """(objective coefficient of x[i, f, j] as coef(f, i, j), or None when the objective has no
        routing term; the coefficient the CPU repair should keep low)."""
        return None, None

    def routing_repair(self, layout):
        """repair(x, z) -> (x', objective change, ok): the incumbent's routing moved within its placement
        until every node's CPU meets the reference checker's absolute tolerance
        (efttc/utils/constraints_step1.py:68-78; core.engine.routing.repair_cpu)."""
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        c0, c1 = layout["c"]
        obj, pref = self.routing_coef()

        def repair(x, z):
            c_open = np.asarray(z[c0:c1], np.float64).reshape(F, N) > 0.5
            room = self.score_room(x, z, layout)
            x2, dpref, ok = repair_cpu(x, d.workload_matrix, d.core_per_req_matrix, d.node_cores_matrix, c_open,
                                       coef=pref, score_room=room)
            dobj = 0.0
            if obj is not None and x2 is not x:
                dobj = dpref if obj is pref else _routing_delta(x, x2, obj)
            return x2, dobj, ok
        return repair

    def score_room(self, x, z, layout):
        """Step 2: rhs + 1e-6 - activity of the score / delay row at (x, z), the room the CPU repair's
        moves may use (None: no such row over x)"""
        return None

    def branch_and_bound(self, model, bmodel=None, **overrides):
        """The step's search (core/engine/bnb.py) over `model` (leaves; max_batch >= batch + 2) and `bmodel`
        (the bound model of bound_model(), or None), configured as solve() runs it; `overrides` replace
        BranchAndBound arguments (the bench's comm / time limit / iteration budgets)."""
        data = self.data
        ub = self.upper_bound()
        layout = model.layout()
        kw = dict(batch=self.batch, tol=self.lp_tol, max_iters=self.lp_max_iters, node_limit=self.node_limit,
                  time_limit=self.time_limit,
                  upper_bound=ub * (1 + 1e-6) + 1e-6 if math.isfinite(ub) else ub, log=self.log,
                  seed_leaves=self.seed_leaves(layout), integer_bound=self.integer_bound(layout),
                  improve=self.improve(layout), repair=self.routing_repair(layout),
                  node_bound_res=self.node_bound_res, unit_flow_leaves=self.unit_flow_leaves,
                  node_max_iters=max(1, int(self.lp_max_iters * self.node_iters_fraction)),
                  bound_lp=bmodel, primal=self.primal_heuristic(layout, _row_map(model)),
                  objective_integral=self.objective_integral(),
                  # step 1: warm starts banded around 8 x the model's cold-start primal weight
                  warm_weight_ref=8.0 if self.step_id() == _lp.STEP1 else 0.0,
                  step2_native=self.native_bound(), branching=self.branching)
        kw.update(overrides)
        return BranchAndBound(model, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix, **kw)

    def solve(self):
        self.init_objective()
        data = self.data
        N, F = len(data.nodes), len(data.functions)
        # `batch` node LPs in flight + one slot for the root's state + one for the incumbent's
        # (core/engine/bnb.py)
        model = make_lp(data, self.VARIANT, self.step_id(), self.batch + 2, **self.model_kwargs())
        bmodel = None
        try:
            bmodel = self.bound_model(data, self.batch + 1)
            res = self.branch_and_bound(model, bmodel).solve()
            layout = model.layout()
        finally:
            model.close()
            if bmodel is not None:
                bmodel.close()
        self.result = res
        if res.objective is not None:
            self._value = float(res.objective)
            self.x_matrix = res.x
            c0, c1 = layout["c"]
            self.c_matrix = np.asarray(res.z[c0:c1], np.float64).reshape(F, N)
            if layout.get("n") is not None:
                self.n_vector = np.asarray(res.z[layout["n"][0]:layout["n"][1]], np.float64)
        else:
            # no feasible placement: the reference reads zeros back from the failed solve
            self._value = 0.0
            self.x_matrix = SparseRouting.empty(N, F)
            self.c_matrix = np.zeros((F, N))
            self.n_vector = np.zeros(N)
        self.log(f"Problem solved with status {res.status} and value {self._value} "
                 f"({res.nodes} nodes, {res.lps} LPs, {res.seconds:.2f}s)")
        return res.status == OPTIMAL

    def results(self):
        self.data.prev_x = self.x_matrix
        self.data.prev_c = self.c_matrix
        return self.x_matrix, self.c_matrix


def _row_map(model):
    """(row_f, row_src) of a model's routing rows (the engine's aggregated rows), or None."""
    rm = getattr(model, "row_map", None)
    return rm() if rm is not None else None


def _max_delay_per_source(data):
    D = np.asarray(data.node_delay_matrix, np.float64)
    return D.max(axis=1)


def _mwd(data):
    """objectives.py:36-43: sum_{f,i} W[f,i] * max{D[i,j'] : D[i,j'] <= maxdelay[f]}, vectorised over the
    distinct max delays."""
    W = np.asarray(data.workload_matrix, np.float64)
    D = np.asarray(data.node_delay_matrix, np.float64)
    md = np.asarray(data.max_delay_matrix, np.float64)
    mwd = 0.0
    for mdv in np.unique(md):
        best = np.where(D <= mdv, D, -np.inf).max(axis=1)
        mwd += float((W[md == mdv] * best[None, :]).sum())
    return mwd


def _routing_delta(x0, x1, coef):
    """sum coef(f, i, j) (x1 - x0) over the loaded rows of two SparseRoutings of one model."""
    tot = 0.0
    for x, s in ((x1, 1.0), (x0, -1.0)):
        f, src = x.row_f[x.row], x.row_src[x.row]
        k = src >= 0
        tot += s * float(np.sum(np.asarray(coef(f[k], src[k], x.dst[k]), np.float64) * x.val[k]))
    return tot


def _delay_coef(data, scale):
    """coef(f, i, j) = scale[f, i] * D[i, j]"""
    D = np.asarray(data.node_delay_matrix, np.float64)
    return lambda f, i, j: scale[f, i] * D[i, j]


class NeptuneStep1CPUBase(NeptuneStepBase):
    pass


class NeptuneStep1CPUMinUtilization(NeptuneStep1CPUBase):
    VARIANT = "MinUtilization"

    def upper_bound(self):
        return float(len(self.data.nodes))

    def objective_weights(self):
        # minimize_utilization (objectives.py:13-28): sum n
        return 1.0, 0.0

    def results(self):
        x, c = super().results()
        self.data.prev_n = self.n_vector
        return x, c


class NeptuneStep1CPUMinDelay(NeptuneStep1CPUBase):
    VARIANT = "MinDelay"

    def upper_bound(self):
        W = np.asarray(self.data.workload_matrix, np.float64)
        return float((W * _max_delay_per_source(self.data)[None, :]).sum())

    def routing_coef(self):
        # minimize_network_delay (objectives.py:4-11): D[i, j] W[f, i]
        c = _delay_coef(self.data, np.asarray(self.data.workload_matrix, np.float64))
        return c, c


class NeptuneStep1CPUMinDelayAndUtilization(NeptuneStep1CPUMinUtilization):
    VARIANT = "MinDelayAndUtilization"

    def __init__(self, alpha=0.5, **kwargs):
        super().__init__(**kwargs)
        self.alpha = alpha

    def load_data(self, data):
        data.alpha = self.alpha
        super().load_data(data)

    def model_kwargs(self):
        return {"alpha": self.alpha}

    def upper_bound(self):
        W = np.asarray(self.data.workload_matrix, np.float64)
        D = np.asarray(self.data.node_delay_matrix, np.float64)
        ub = float(self.alpha)
        if W.sum():
            mwd = _mwd(self.data)
            if mwd > 0:
                ub += (1 - self.alpha) * float((W * D.max(axis=1)[None, :]).sum()) / mwd
        return ub

    def objective_weights(self):
        # minimize_node_delay_and_utilization (objectives.py:30-53): alpha / N per open node, (1 - alpha) / MWD
        W = np.asarray(self.data.workload_matrix, np.float64)
        mwd = _mwd(self.data) if W.sum() else 0.0
        return self.alpha / len(self.data.nodes), ((1 - self.alpha) / mwd if mwd > 0 else 0.0)

    def routing_coef(self):
        # minimize_node_delay_and_utilization (objectives.py:30-53): (1 - alpha) W[f, i] D[i, j] / MWD, no x
        # terms when sum W = 0
        W = np.asarray(self.data.workload_matrix, np.float64)
        mwd = _mwd(self.data) if W.sum() else 0.0
        if mwd <= 0:
            return None, None
        c = _delay_coef(self.data, (1 - self.alpha) * W / mwd)
        return c, c


class NeptuneStep2Base(NeptuneStepBase):
    node_bound_res = 0.0   # every node LP to its certificate (see NeptuneStepBase.node_bound_res)
    unit_flow_leaves = False
    node_iters_fraction = 1.0
    branching = 0

    def __init__(self, mode=str, soften_step1_sol=1.3, **kwargs):
        super().__init__(**kwargs)
        self.mode = mode
        assert mode in ["delete", "create"]
        self.soften_step1_sol = soften_step1_sol

    def step_id(self):
        return _lp.STEP2_DELETE if self.mode == "delete" else _lp.STEP2_CREATE

    def model_kwargs(self):
        d = self.data
        kw = {"soften_step1_sol": self.soften_step1_sol, "max_score": float(getattr(d, "max_score", 0.0) or 0.0)}
        prev = getattr(d, "prev_x", None)
        if prev is not None and np.size(prev):
            # constraints_step2.py:66-68: sum D[i,j] W[f,i] prev_x[i,f,j]
            D = np.asarray(d.node_delay_matrix, np.float64)
            W = np.asarray(d.workload_matrix, np.float64)
            if isinstance(prev, SparseRouting):
                kw["prev_network_delay"] = prev.network_delay(D, W)
            else:
                kw["prev_network_delay"] = float(np.einsum("ij,fi,ifj->", D, W, np.asarray(prev, np.float64)))
        return kw

    def upper_bound(self):
        # minimize_disruption (objectives.py:55-63): w * sum(moved) with at most one move per (f, j),
        # allocated / deallocated <= 0
        FN = len(self.data.nodes) * len(self.data.functions)
        return float(FN) * FN

    def seed_leaves(self, layout):
        """Step 2's natural primal starts (neptune.py:18-30): the step-1 placement (it meets the
        score row by construction) and the old allocation (no moves)."""
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        c0, c1 = layout["c"]
        cands = []
        prev = getattr(d, "prev_c", None)
        if prev is not None and np.size(prev) == F * N:
            cands.append((np.asarray(prev, np.float64).reshape(F, N) > 0.5).astype(np.float64))
        old = np.asarray(d.old_allocations_matrix, np.float64).reshape(F, N)
        cands.append((old > 0.5).astype(np.float64))
        out = []
        for c in cands:
            if (c.sum(axis=1) < 1).any():
                continue
            idx, val = [np.arange(c0, c1)], [c.ravel()]
            if layout.get("n") is not None:
                n0, n1 = layout["n"]
                idx.append(np.arange(n0, n1))
                val.append((c.sum(axis=0) >= 1).astype(np.float64))
            out.append((np.concatenate(idx), np.concatenate(val)))
        return out

    def node_cap(self):
        """The most nodes an integral step-2 placement can open (n binary, n = 1 wherever c = 1 by
        C6/C7), from the step-2 rows on n: MinUtilization's sum n <= max_score * soften
        (constraints_step2.py:71-73); MinDelayAndUtilization's score row (:76-88), whose x terms are
        >= 0, gives alpha / N * sum n <= max_score * soften.  inf when nothing caps it."""
        if self.VARIANT not in ("MinUtilization", "MinDelayAndUtilization"):
            return math.inf
        d = self.data
        ms = float(getattr(d, "max_score", 0.0) or 0.0) * self.soften_step1_sol
        if self.VARIANT == "MinUtilization":
            return ms
        if self.score_row_lower_bound() > ms * (1 + 1e-9) + 1e-9:
            return -1.0          # no integral placement meets the score row: every box's integer bound is +inf
        return ms * len(d.nodes) / self.alpha if self.alpha > 0 else math.inf

    def score_row_lower_bound(self):
        """A lower bound on the MinDelayAndUtilization score row (constraints_step2.py:76-88)
        alpha / N sum n + sum (1 - alpha) W[f,i] D[i,j] / MD[i,f] x[i,f,j] over every INTEGRAL placement of this
        step (MD[i,f] = max(maxdelay[f], max_k D[k,i]), :77-81).  A loaded source i of f routes at no delay only to
        j = i (D[i,i] = 0), which needs c[f,i] = 1 (C1); any other destination costs at least g[f,i] = (1 - alpha)
        W[f,i] dmin[i] / MD[i,f], dmin[i] = min_{j != i} D[i,j].  With k open nodes at most the pairs of k nodes are
        local, and in delete mode (D4, sum c <= sum old) at most sum old pairs: so
          score >= min_k  alpha k / N + sum g - min(top_k(node sums of g), top_{sum old}(g))   (k >= 1).
        +0 when it proves nothing.  On the SURVEY §8(d) generator the bound exceeds 1.3 x the step-1 score at every
        size (64x32: 0.477 create / 7.55 delete against 0.177), so both step-2 modes are proven infeasible before any
        LP — the reference's SCIP returns INFEASIBLE for the same models (neptune.py:24-39 then keeps step 1)."""
        if self.VARIANT != "MinDelayAndUtilization":
            return 0.0
        d = self.data
        W = np.asarray(d.workload_matrix, np.float64)
        if not W.any():
            return 0.0
        D = np.asarray(d.node_delay_matrix, np.float64)
        F, N = W.shape
        md = np.maximum(np.asarray(d.max_delay_matrix, np.float64)[None, :], D.max(axis=0)[:, None])   # [i, f]
        off = D + np.diag(np.full(N, np.inf))
        dmin = off.min(axis=1) if N > 1 else np.zeros(N)
        g = (1 - self.alpha) * W * dmin[None, :] / md.T                                                  # [f, i]
        tot = float(g.sum())
        cum = np.concatenate([[0.0], np.cumsum(np.sort(g.sum(axis=0))[::-1])])
        k = np.arange(1, N + 1)
        local = cum[k]
        if self.mode == "delete":
            O = int(round(float((np.asarray(d.old_allocations_matrix, np.float64) > 0.5).sum())))
            local = np.minimum(local, float(np.sort(g.ravel())[::-1][:O].sum()))
        return max(0.0, float(np.min(self.alpha / N * k + tot - local)))

    def native_bound(self):
        """(create, node cap, old allocation): integer_bound below, evaluated by the native tree
        (csrc/nep_bnb.cpp NepBnb::ibound, the same closed form)."""
        return (self.mode == "create", float(self.node_cap()),
                np.asarray(self.data.old_allocations_matrix, np.float64).reshape(-1))

    def integer_bound(self, layout=None):
        """The step-2 objective over integral placements, bounded from the node's c (and n) fixings.

        With c binary, A = #(c=1, old=0) additions, R = #(c=0, old=1) removals and O = sum old,
        minimize_disruption (objectives.py:55-63, w = F*N) under constrain_migrations
        (constraints_step2.py:19-33) is w(A+R) + (w-1) allocated + (w+1) deallocated with
          create (:47-54): sum c >= O and the optimum A + (2w-1) R,
          delete (:36-44): sum c <= O and the optimum (2w+1) A - R.
        Every function needs an open destination (constraints_step1.py:27-35 with :5-15: its rows
        route somewhere and c >= flow / M), so A is at least the fixed additions plus one per
        function that no fixed-1 c and no free old c can cover.  The bound is the closed form at
        those least A, R (largest R for delete), +inf when the sum-c condition cannot hold.
        With at most K nodes open (node_cap), the old allocations kept sit on at most K nodes:
        R >= O - (the most keepable old entries on K nodes that include every node the fixings open)."""
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        FN = F * N
        w = float(FN)
        old = (np.asarray(d.old_allocations_matrix, np.float64).reshape(FN) > 0.5)
        O = float(old.sum())
        create = self.mode == "create"
        K = self.node_cap()
        Kint = math.floor(K + 1e-9) if math.isfinite(K) else None
        nr = None if layout is None else layout.get("n")

        def bound(idx, val):
            fx = np.full(FN, -1.0)
            sel = idx < FN                                    # c occupies z_int[0 : F*N] (neptune_lp.h)
            fx[idx[sel]] = val[sel]
            one, zero = fx > 0.5, (fx >= 0) & (fx < 0.5)
            add_fixed = float((one & ~old).sum())
            rem_fixed = float((zero & old).sum())
            covered = (one | (old & ~zero)).reshape(F, N).any(axis=1)
            A = add_fixed + float((~covered).sum())
            R_lb = rem_fixed
            if Kint is not None:
                nf = np.full(N, -1.0)
                if nr is not None:
                    seln = (idx >= nr[0]) & (idx < nr[1])
                    nf[idx[seln] - nr[0]] = val[seln]
                opened = (nf > 0.5) | one.reshape(F, N).any(axis=0)
                closed = (nf >= 0) & (nf < 0.5)
                if (opened & closed).any() or opened.sum() > Kint:
                    return math.inf
                keep = ((old & ~zero).reshape(F, N).sum(axis=0)).astype(np.float64)
                keep[closed] = 0.0
                free = np.sort(keep[~opened & ~closed])[::-1]
                best = float(keep[opened].sum()) + float(free[:max(0, Kint - int(opened.sum()))].sum())
                R_lb = max(R_lb, O - best)
                # additions: a function with no placement fixed open needs one, and it costs no addition only
                # on an open node where it has an old placement (not closed) — at most K nodes hold those, so
                # at most the K best nodes' counts of such functions (the forced-open ones included) avoid one
                freef = ~one.reshape(F, N).any(axis=1)
                cov = ((old & ~zero).reshape(F, N) & freef[:, None]).sum(axis=0).astype(np.float64)
                cov[closed] = 0.0
                rest = np.sort(cov[~opened & ~closed])[::-1]
                cover = float(cov[opened].sum()) + float(rest[:max(0, Kint - int(opened.sum()))].sum())
                A = max(A, add_fixed + max(0.0, float(freef.sum()) - cover))
            if create:
                if FN - float(zero.sum()) < O:
                    return math.inf
                return A + (2 * w - 1) * R_lb
            ones_f = one.reshape(F, N).sum(axis=1)
            if float(np.maximum(ones_f, 1.0).sum()) > O + 1e-9:
                return math.inf
            # R = O - kept: the fixed-open old placements are kept, and so is one old placement of every function
            # without a fixed placement that needs no addition (at most A - add_fixed of them need one)
            nfree = float((ones_f == 0).sum())
            kept = float((one & old).sum()) + max(0.0, nfree - (A - add_fixed))
            return (2 * w + 1) * A - (O - kept)
        return bound

    def improve(self, layout, top=4):
        """Node relocation around a new incumbent: exchange the placement columns of two nodes
        (c[:, ju] <-> c[:, jt], n alike), for every node ju the incumbent uses and every other node jt.
        The step-2 objective depends on c only (integer_bound's closed form in A, R), so every
        exchange is priced exactly from column counts (A(p, o) = p . (1 - o), R(p, o) = (1 - p) . o,
        one F x N by N x F product each); sum c is unchanged (D3/D4 hold as before), memory (C3,
        constraints_step1.py:18-23) is checked, and the `top` cheapest exchanges below the incumbent
        are returned as leaves (their LPs re-check routing and the remaining rows).  E.g. the Alibaba
        MDU case: step 1 puts every function on one node, step 2 must keep one node (score row) and
        the optimum is the node holding most of the old allocation."""
        d = self.data
        F, N = len(d.functions), len(d.nodes)
        FN = F * N
        old = (np.asarray(d.old_allocations_matrix, np.float64).reshape(F, N) > 0.5).astype(np.float64)
        mem_f = np.asarray(d.function_memory_matrix, np.float64).reshape(F)
        node_mem = np.asarray(d.node_memory_matrix, np.float64).reshape(N)
        w = float(FN)
        ka, kr = (1.0, 2 * w - 1) if self.mode == "create" else (2 * w + 1, -1.0)
        has_n = layout.get("n") is not None

        def neighbours(idx, val, value):
            c = np.zeros(FN)
            sel = idx < FN
            c[idx[sel]] = val[sel]
            P = (c.reshape(F, N) > 0.5).astype(np.float64)
            Acol = (P * (1 - old)).sum(axis=0)                 # additions per node
            Rcol = ((1 - P) * old).sum(axis=0)                 # removals per node
            Across = P.T @ (1 - old)                           # [a, b]: column a's pattern on node b
            Rcross = (1 - P).T @ old
            used = np.flatnonzero(P.sum(axis=0) > 0)
            if used.size == 0:
                return []
            memcol = mem_f @ P                                 # memory of each column's pattern
            dA = Across[used, :] + Across[:, used].T - Acol[used][:, None] - Acol[None, :]
            dR = Rcross[used, :] + Rcross[:, used].T - Rcol[used][:, None] - Rcol[None, :]
            delta = ka * dA + kr * dR                          # objective change of exchanging (ju, jt)
            ok = (memcol[used][:, None] <= node_mem[None, :] + 1e-9) & (memcol[None, :] <= node_mem[used][:, None] + 1e-9)
            ok &= used[:, None] != np.arange(N)[None, :]
            delta = np.where(ok, delta, np.inf)
            order = np.argsort(delta, axis=None, kind="stable")[:top]
            out = []
            for k in order:
                if not delta.flat[k] < -0.5:                     # integral objective: improve by >= 1
                    break
                u, t = divmod(int(k), N)
                ju = int(used[u])
                Q = P.copy()
                Q[:, [ju, t]] = Q[:, [t, ju]]
                ids, vs = [np.arange(FN)], [Q.ravel()]
                if has_n:
                    n0, n1 = layout["n"]
                    ids.append(np.arange(n0, n1))
                    vs.append((Q.sum(axis=0) > 0).astype(np.float64))
                out.append((np.concatenate(ids), np.concatenate(vs)))
            return out
        return neighbours

    def routing_coef(self):
        # minimize_disruption (objectives.py:55-63) has no routing term; moves prefer lowering the score
        # row: D6 (MinDelay, constraints_step2.py:57-69) D[i, j] W[f, i], D7 (MinDelayAndUtilization, :76-88)
        # (1 - alpha) W[f, i] D[i, j] / max(maxdelay[f], max_k D[k, i]); MinUtilization's D5 has no x
        d = self.data
        W = np.asarray(d.workload_matrix, np.float64)
        if self.VARIANT == "MinDelay":
            return None, _delay_coef(d, W)
        if self.VARIANT == "MinDelayAndUtilization":
            D = np.asarray(d.node_delay_matrix, np.float64)
            md = np.maximum(np.asarray(d.max_delay_matrix, np.float64)[:, None], D.max(axis=0)[None, :])   # [f, i]
            return None, _delay_coef(d, (1 - self.alpha) * W / md)
        return None, None

    def score_room(self, x, z, layout):
        # D6 (MinDelay, constraints_step2.py:57-69): sum D W x <= soften * prev delay; D7 (MDU, :76-88):
        # alpha / N sum n + sum (1 - alpha) W D / max(maxdelay, max_k D[k, i]) x <= soften * max_score;
        # the checker allows + 1e-6 (efttc/utils/constraints_step2.py:68, :95).  D5 (MU) has no x.
        _, pref = self.routing_coef()
        if pref is None:
            return None
        d = self.data
        i, f, j, v = x.entries() if hasattr(x, "entries") else SparseRouting.from_dense(x).entries()
        act = float(np.sum(np.asarray(pref(f, i, j), np.float64) * v))
        if self.VARIANT == "MinDelay":
            rhs = self.soften_step1_sol * self.model_kwargs().get("prev_network_delay", 0.0)
        else:
            rhs = float(getattr(d, "max_score", 0.0) or 0.0) * self.soften_step1_sol
            nr = layout.get("n")
            if nr is not None:
                act += self.alpha / len(d.nodes) * float(np.sum(np.asarray(z[nr[0]:nr[1]], np.float64)))
        return rhs + 1e-6 - act

    def results(self):
        # neptune_step2.py:43-51: no side effects on data (the prints are logs only)
        return self.x_matrix, self.c_matrix


class NeptuneStep2MinUtilization(NeptuneStep2Base):
    VARIANT = "MinUtilization"


class NeptuneStep2MinDelay(NeptuneStep2Base):
    VARIANT = "MinDelay"


class NeptuneStep2MinDelayAndUtilization(NeptuneStep2MinUtilization):
    VARIANT = "MinDelayAndUtilization"

    def __init__(self, alpha=0.5, **kwargs):
        super().__init__(**kwargs)
        self.alpha = alpha

    def model_kwargs(self):
        kw = super().model_kwargs()
        kw["alpha"] = self.alpha
        return kw
