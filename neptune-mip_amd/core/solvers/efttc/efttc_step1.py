"""EF-TTC step 1: the Top-Trading-Cycles placement heuristic (reference
`core/solvers/efttc/efttc_step1.py:7-441`), restated over numpy state.

It is not an LP and not on the GPU path: NEPTUNE uses it only as the step 1 of the
`NeptuneWithEFTTC*` solvers (reference `core/solvers/neptune/neptune.py:68-93`), whose step 2 is the
NEPTUNE MIP on the MI355X engine, and as the `Efttc*` solvers.  Every decision follows the
reference exactly — preference ranking with the (score, index) tie-break (:123-146), the cycle walk
(:148-185), the per-cycle memory / CPU / budget checks, snapshot-restore and invalid-pair rules
(:48-121, :240-268) and the delay-improvement test (:197-238) — so placements, scores and the errors
it raises (e.g. the KeyError of :115 when one cycle lists a function twice) are the reference's.

State: x[i, f, j] float64, c[f, j] bool, n[j] bool (the reference's {"val": ...} dicts).
"""
import numpy as np

from ..solver import Solver
from . import scoring


class EfttcStepBase(Solver):
    OBJECTIVE = "min_delay_min_utilization"

    def __init__(self, **kwargs):
        self.invalid_pairs = set()
        super().__init__(**kwargs)
        self.x = self.c = self.n = None
        self.objective = self.OBJECTIVE

    # reference variables.py:4-17
    def init_vars(self):
        N, F = len(self.data.nodes), len(self.data.functions)
        self.x = np.zeros((N, F, N))
        self.c = np.zeros((F, N), bool)
        self.n = np.zeros(N, bool)

    def init_constraints(self):
        pass

    def get_constraints(self):
        return True

    def snapshot_vars(self):
        return self.x.copy(), self.c.copy(), self.n.copy()

    def restore_vars(self, snap):
        self.x, self.c, self.n = snap[0].copy(), snap[1].copy(), snap[2].copy()

    # ------------------------------------------------------------------------------------------
    def solve(self):
        self.init_vars()
        remaining_functions = set(range(len(self.data.functions)))
        remaining_nodes = set(range(len(self.data.nodes)))
        tried_cycles = set()
        while remaining_functions:
            graph = self.build_preference_graph(remaining_functions, remaining_nodes)
            cycle = self.find_cycle(graph)
            if not cycle:
                break
            key = tuple(sorted(cycle))
            if key in tried_cycles:
                break
            snap = self.snapshot_vars()
            if not self.can_assign_cycle(cycle):
                tried_cycles.add(key)
                continue
            if self.get_constraints():
                self.handle_cycle(cycle, remaining_functions, remaining_nodes, snap)
            else:
                tried_cycles.add(key)
                self.restore_vars(snap)
                self.invalid_pairs.update(cycle)

    def _mem_used(self, j):
        fm = self.data.function_memory_matrix
        return sum(fm[f2] if self.c[f2, j] else 0 for f2 in range(len(self.data.functions)))

    def handle_cycle(self, cycle, remaining_functions, remaining_nodes, snap):
        # reference :99-121, including its loop structure: the inner loops run once per pair of the
        # cycle, so a function listed twice is removed twice (set.remove raises KeyError, as there)
        node_mem = self.data.node_memory_matrix
        for _, j in cycle:
            used = self._mem_used(j)
            if used == node_mem[j]:
                remaining_nodes.discard(j)
            if used > node_mem[j]:
                self.restore_vars(snap)
                self.invalid_pairs.update(cycle)
            else:
                self.invalid_pairs.update(cycle)
                if "min_delay" in self.objective:
                    for f, _ in cycle:
                        if self.find_best_node_by_delay_improvement(f, remaining_nodes) is None:
                            remaining_functions.remove(f)
                else:
                    for f, _ in cycle:
                        remaining_functions.discard(f)

    def build_preference_graph(self, remaining_functions, remaining_nodes):
        graph = {}
        for f in remaining_functions:
            pref = self.rank_nodes_for_function(f, remaining_nodes)
            if pref:
                graph[f] = ~pref[0]
        for j in remaining_nodes:
            pref = self.rank_functions_for_node(j, remaining_functions)
            if pref:
                graph[~j] = pref[0]
        return graph

    def rank_nodes_for_function(self, f, node_pool):
        valid = [j for j in node_pool if (f, j) not in self.invalid_pairs]
        return sorted(valid, key=lambda j: (self.score_local(f, j), abs(j)))

    def rank_functions_for_node(self, j, function_pool):
        return sorted(function_pool, key=lambda f: (self.score_local(f, j), abs(f)))

    @staticmethod
    def find_cycle(graph):
        """First cycle of the functional graph (functions f >= 0, nodes ~j < 0) in the order the
        walk meets it; returned as (function, node) pairs."""
        visited = set()
        for start in graph:
            if start in visited:
                continue
            path, seen, cur = [], set(), start
            while cur not in seen:
                seen.add(cur)
                path.append(cur)
                if cur not in graph:
                    break
                nxt = graph[cur]
                path.append(nxt)
                if nxt in seen:
                    k = path.index(nxt)
                    out, dup = [], set()
                    for a, b in zip(path[k:-1], path[k + 1:]):
                        if a >= 0 and b < 0:
                            pair = (a, ~b)
                        elif a < 0 and b >= 0:
                            pair = (b, ~a)
                        else:
                            continue
                        if pair not in dup:
                            dup.add(pair)
                            out.append(pair)
                    return out
                cur = nxt
            visited |= seen
        return []

    def change_n_one(self, j):
        self.n[j] = bool(self.c[:, j].any())

    def change_x_one(self, f):
        """Every source routes f to its nearest active destinations, split evenly (:187-195)."""
        active = [j for j in range(len(self.data.nodes)) if self.c[f, j]]
        if not active:
            return
        D = self.data.node_delay_matrix
        for i in range(len(self.data.nodes)):
            d = {j: D[i][j] for j in active}
            dmin = min(d.values())
            best = [j for j, v in d.items() if abs(v - dmin) < 1e-6]
            val = 1.0 / len(best)
            for j in active:
                self.x[i, f, j] = val if j in best else 0.0

    def find_best_node_by_delay_improvement(self, f, candidate_nodes):
        if not candidate_nodes:
            return None
        useful = [j for j in candidate_nodes if not self.c[f, j] and (f, j) not in self.invalid_pairs]
        if not useful:
            return None
        data = self.data
        wf = data.workload_matrix[f]
        D = data.node_delay_matrix
        active = [j2 for j2 in range(len(data.nodes)) if self.c[f, j2]]
        cur_vec = np.min(D[:, active], axis=1) if active else np.full(len(data.nodes), np.inf)
        cur_score = np.sum(wf * cur_vec)
        best_node, best_delta = None, 0.0
        for j in useful:
            new_vec = np.minimum(cur_vec, D[:, j])
            delta = cur_score - np.sum(wf * new_vec)
            if self.objective == "min_delay":
                if delta > best_delta + 1e-6:
                    best_delta, best_node = delta, j
            elif self.objective == "min_delay_min_utilization":
                alpha = getattr(data, "alpha", 0.5)
                du = (1 / len(data.nodes)) if not self.n[j] else 0
                ds = (1 - alpha) * delta - alpha * du
                if ds > best_delta + 1e-6:
                    best_delta, best_node = ds, j
        return best_node

    def can_assign_cycle(self, cycle):
        ok = False
        for f, j in cycle:
            if not self.can_assign(f, j):
                self.invalid_pairs.add((f, j))
                continue
            self.c[f, j] = True
            self.change_x_one(f)
            self.change_n_one(j)
            ok = True
        return ok

    def can_assign(self, f, j):
        return self._mem_used(j) + self.data.function_memory_matrix[f] <= self.data.node_memory_matrix[j]

    def score_local(self, f, j):
        raise NotImplementedError("Efttc must implement score_local(f, j)")

    def get_objective(self):
        raise NotImplementedError("Efttc must implement get_objective()")

    def results(self):
        """x[i, f, j], c[f, j] as float matrices (reference efttc/utils/output.py:5-16)."""
        return self.x.astype(np.float64), self.c.astype(np.float64)

    def score(self):
        return self.get_objective()


class EfttcStep1CPUBase(EfttcStepBase):
    def get_constraints(self):
        # reference :306-318: the handle-all-requests check is disabled there; CPU stays
        return super().get_constraints() and scoring.cpu_usage_ok(self.data, self.x)


class EfttcStep1CPUMinUtilization(EfttcStep1CPUBase):
    OBJECTIVE = "min_utilization"

    def get_constraints(self):
        return super().get_constraints() and scoring.budget_ok(self.data, self.n)

    def get_objective(self):
        return scoring.node_utilization(self.data, self.n)

    def score_local(self, f, j):
        planned = int(self.c[:, j].sum())
        old = self.data.old_allocations_matrix
        bonus, actual = 1.0, 0
        if isinstance(old, np.ndarray):
            bonus = 0.5 if old[f, j] else 1.0
            actual = int(np.sum(old[:, j]))
        return (self.data.node_costs[j] / (1 + planned + actual)) * bonus

    def results(self):
        x, c = super().results()
        self.data.prev_n = self.n.astype(np.float64)
        self.data.prev_x = x
        self.data.prev_c = c
        return x, c


class EfttcStep1CPUMinDelay(EfttcStep1CPUBase):
    OBJECTIVE = "min_delay"

    def get_objective(self):
        return scoring.network_delay(self.data, self.x)

    def score_local(self, f, j):
        d = self.data.node_delay_matrix[:, j].dot(self.data.workload_matrix[f])
        return d * (0.5 if self.data.old_allocations_matrix[f, j] == 1 else 1.0)


class EfttcStep1CPUMinDelayAndUtilization(EfttcStep1CPUMinUtilization):
    OBJECTIVE = "min_delay_min_utilization"

    def __init__(self, alpha=0.5, **kwargs):
        super().__init__(**kwargs)
        self.alpha = alpha

    def load_data(self, data):
        data.alpha = self.alpha
        super().load_data(data)

    def get_objective(self):
        return scoring.node_delay_and_utilization(self.data, self.n, self.x, self.alpha)

    def score_local(self, f, j):
        bonus = 0.5 if (self.data.old_allocations_matrix is not None and self.data.old_allocations_matrix[f, j] == 1) \
            else 1.0
        util = int(self.c[:, j].sum())
        delay = np.dot(self.data.node_delay_matrix[:, j], self.data.workload_matrix[f])
        return (self.alpha * (self.data.node_costs[j] / (1 + util)) + (1 - self.alpha) * delay) * bonus
