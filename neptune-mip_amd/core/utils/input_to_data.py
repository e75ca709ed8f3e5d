"""Payload -> `Data` (reference: `core/utils/input_to_data.py`).

Semantics kept from the reference (line refs into its input_to_data.py):
  * required keys and consistency asserts (check_input :46-86) -> AssertionError (HTTP 500)
  * delay matrix defaults to 0 on the diagonal / 1 elsewhere (:152-156); workload, workload on
    destination and cores matrices default to zeros (:159-178)
  * every function's max delay is 1000 regardless of `function_max_delays` (:136)
  * function keys match on name.split('/')[1] (:199, :269)
  * core_per_req = nan_to_num(cores / workload_on_destination, nan=0): x/0 -> inf -> max float (:272)
  * the old CPU allocation is all ones when the request carries none (:274-276)
  * node cost 5, budget 300 (:185-187)
The metrics-database path (`with_db=True`, :206-262, a Kubernetes PostgreSQL) is out of scope and
raises NotImplementedError.
"""
import numpy as np

from .data import Data

REQUIRED_KEYS = ("community", "namespace", "function_names", "function_memories", "gpu_function_names",
                 "gpu_function_memories", "node_names", "node_memories", "node_cores", "gpu_node_names",
                 "gpu_node_memories", "function_max_delays", "actual_cpu_allocations", "actual_gpu_allocations")

NODE_COST = 5
NODE_BUDGET = 300
FUNCTION_MAX_DELAY = 1000


def check_input(schedule_input):
    missing = [k for k in REQUIRED_KEYS if k not in schedule_input]
    assert not missing, f"Key `{missing[0]}` not in schedule input"
    g = schedule_input.get
    assert set(g("gpu_function_names", [])) <= set(g("function_names", [])), "GPU functions must be functions"
    assert len(g("function_names", [])) == len(g("function_memories", [])), "function_names / function_memories"
    assert len(g("gpu_function_names", [])) == len(g("gpu_function_memories", [])), "gpu function memories"
    assert set(g("gpu_node_names", [])) <= set(g("node_names", [])), "GPU nodes must be nodes"
    assert len(g("node_names", [])) == len(g("node_memories", [])), "node_names / node_memories"
    assert len(g("gpu_node_names", [])) == len(g("gpu_node_memories", [])), "gpu node memories"


def _matrix_or(payload, key, shape, fill):
    value = payload.get(key, None)
    if value:
        return np.array(value)
    return np.full(shape, fill, dtype=np.int64)


def data_to_solver_input(payload, workload_coeff=1, with_db=True):
    if with_db:
        raise NotImplementedError("with_db=True reads the NEPTUNE metrics database "
                                  "(reference input_to_data.py:206-262); out of scope — send with_db=false")
    nodes = list(payload.get("node_names", []))
    functions = list(payload.get("function_names", []))
    N, F = len(nodes), len(functions)
    data = Data(nodes, functions)
    data.node_memory_matrix = np.array(payload.get("node_memories"))
    data.function_memory_matrix = np.array(payload.get("function_memories"))
    data.node_delay_matrix = _matrix_or(payload, "node_delay_matrix", (N, N), 1)
    if not payload.get("node_delay_matrix", None):
        np.fill_diagonal(data.node_delay_matrix, 0)
    data.workload_matrix = _matrix_or(payload, "workload_on_source_matrix", (F, N), 0) * workload_coeff
    w_dest = _matrix_or(payload, "workload_on_destination_matrix", (F, N), 0)
    data.cores_matrix = _matrix_or(payload, "cores_matrix", (F, N), 0)
    data.max_delay_matrix = np.full(F, FUNCTION_MAX_DELAY)
    data.response_time_matrix = np.zeros((F, N), np.int64)
    data.node_cores_matrix = np.array(payload.get("node_cores"))
    with np.errstate(divide="ignore", invalid="ignore"):
        data.core_per_req_matrix = np.nan_to_num(data.cores_matrix / w_dest, nan=0)

    node_pos = {name: k for k, name in enumerate(nodes)}
    fn_pos = {}
    for k, name in enumerate(functions):
        fn_pos[name.split("/")[1]] = k
    old = np.zeros((F, N), np.int64)
    for fn_key, placement in payload.get("actual_cpu_allocations", {}).items():
        if not placement:
            continue
        row = fn_pos[fn_key.split("/")[1]]
        for node, flag in placement.items():
            old[row, node_pos[node]] = flag
    old = (old != 0).astype(np.int64)
    data.old_allocations_matrix = old if old.any() else np.ones_like(old)
    data.node_costs = np.full(N, NODE_COST)
    data.node_budget = NODE_BUDGET
    return data
