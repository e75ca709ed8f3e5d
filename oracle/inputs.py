"""ORACLE (test infrastructure only): restatement of the reference's payload tensorisation.

Follows `core/utils/input_to_data.py` of the reference:
  check_input             :46-86
  data_to_solver_input    :88-111   (DB path :206-262 is out of scope -> NotImplementedError)
  setup_community_data    :114-136  (max delay forced to 1000 per function, :136)
  setup_runtime_data      :151-183  (D default: 0 on the diagonal, 1 elsewhere, :156)
  setup_budget_data       :185-187  (cost 5 per node, budget 300)
  create_mappings         :189-203  (function key = name.split('/')[1], :199)
  update_old_allocations  :265-286  (cores/wdest with nan->0, inf->max float :272;
                                     all-ones old allocation when empty :275-276)
"""
from types import SimpleNamespace

import numpy as np

REQUIRED_KEYS = ("community", "namespace", "function_names", "function_memories", "gpu_function_names",
                 "gpu_function_memories", "node_names", "node_memories", "node_cores", "gpu_node_names",
                 "gpu_node_memories", "function_max_delays", "actual_cpu_allocations", "actual_gpu_allocations")


def check_input(payload):
    """input_to_data.py:46-86 — raises AssertionError exactly where the reference does."""
    for k in REQUIRED_KEYS:
        assert k in payload, f"Key `{k}` not in schedule input"
    fns, gfns = payload.get("function_names", []), payload.get("gpu_function_names", [])
    assert set(gfns).issubset(set(fns))
    assert len(fns) == len(payload.get("function_memories", []))
    assert len(gfns) == len(payload.get("gpu_function_memories", []))
    nodes, gnodes = payload.get("node_names", []), payload.get("gpu_node_names", [])
    assert set(gnodes).issubset(set(nodes))
    assert len(nodes) == len(payload.get("node_memories", []))
    assert len(gnodes) == len(payload.get("gpu_node_memories", []))


def data_to_solver_input(payload, workload_coeff=1, with_db=True):
    if with_db:
        raise NotImplementedError("metrics-DB path (input_to_data.py:206-262) is out of scope")
    nodes = list(payload.get("node_names", []))
    functions = list(payload.get("function_names", []))
    N, F = len(nodes), len(functions)

    dm = payload.get("node_delay_matrix", None)
    D = np.array(dm) if dm else (1 - np.eye(N, dtype=np.int64))
    ws = payload.get("workload_on_source_matrix", None)
    W = np.array(ws) if ws else np.zeros((F, N), np.int64)
    wd = payload.get("workload_on_destination_matrix", None)
    wdest = np.array(wd) if wd else np.zeros((F, N), np.int64)
    cm = payload.get("cores_matrix", None)
    cores_m = np.array(cm) if cm else np.zeros((F, N), np.int64)

    node_idx = {n: i for i, n in enumerate(nodes)}
    fn_idx = {}
    for i, fn in enumerate(functions):
        fn_idx[fn.split("/")[1]] = i
    old = np.zeros((F, N), np.int64)
    for key, per_node in payload.get("actual_cpu_allocations", {}).items():
        for node, ok in per_node.items():
            if per_node:
                old[fn_idx[key.split("/")[1]]][node_idx[node]] = ok
    with np.errstate(divide="ignore", invalid="ignore"):
        cpr = np.nan_to_num(cores_m / wdest, nan=0)
    old = old.astype(bool).astype(np.int64)
    if old.sum() == 0:
        old = old + 1

    return SimpleNamespace(
        nodes=nodes, functions=functions,
        node_memory_matrix=np.array(payload.get("node_memories")),
        function_memory_matrix=np.array(payload.get("function_memories")),
        node_delay_matrix=D,
        workload_matrix=W * workload_coeff,
        max_delay_matrix=np.array([1000] * F),
        node_cores_matrix=np.array(payload.get("node_cores")),
        cores_matrix=cores_m,
        old_allocations_matrix=old,
        core_per_req_matrix=cpr,
        node_costs=np.array([5] * N),
        node_budget=300,
        prev_x=np.array([]),
    )
