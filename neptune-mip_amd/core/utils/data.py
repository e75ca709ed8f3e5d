"""`Data` — the tensors one scheduling request is turned into (reference: `core/utils/data.py:5-26`).

Same attribute names as the reference so existing callers (main.py, the score-analysis scripts)
keep working.  Shapes: nodes N, functions F.
  node_memory_matrix [N], function_memory_matrix [F], node_delay_matrix [N,N] D[i,j],
  workload_matrix [F,N] W[f,i], max_delay_matrix [F], node_cores_matrix [N], cores_matrix [F,N],
  core_per_req_matrix [F,N], old_allocations_matrix [F,N] (0/1), node_costs [N], node_budget.
  prev_x: empty until a step-1 solve wrote x[i,f,j] (the reference's "no GPU step" sentinel).
Solvers also attach prev_c, prev_n, max_score and alpha while they run (neptune_step1.py:21-27,73,
neptune.py:22).
"""
from typing import List, Optional

import numpy as np


class Data:
    def __init__(self, nodes: Optional[List[str]] = None, functions: Optional[List[str]] = None):
        self.nodes = list(nodes) if nodes else []
        self.functions = list(functions) if functions else []
        empty = np.array([])
        for name in ("node_memory_matrix", "function_memory_matrix", "node_delay_matrix", "workload_matrix",
                     "max_delay_matrix", "response_time_matrix", "node_cores_matrix", "cores_matrix",
                     "old_allocations_matrix", "core_per_req_matrix", "gpu_function_memory_matrix",
                     "gpu_node_memory_matrix", "prev_x", "node_costs"):
            setattr(self, name, empty)
        self.node_budget = 0

    @property
    def shape(self):
        return len(self.nodes), len(self.functions)

    def __repr__(self):
        return f"Data(N={len(self.nodes)}, F={len(self.functions)})"
