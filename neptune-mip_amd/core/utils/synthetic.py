"""Seeded synthetic NEPTUNE payloads (SURVEY.md §8(d) "Configs as concrete synthetic inputs").

The reference has no generator for its large shapes: its inputs come from the REST
payload (`main.py:31-51`) or the Alibaba trace (`testing/alibaba/build_dataset_alibaba.py`,
whose raw trace is absent).  These generators emit *REST payloads* (the dict that
`check_input` / `data_to_solver_input` consume, `core/utils/input_to_data.py:46-111`)
so the very same bytes drive the CPU oracle and the GPU path.

`synthetic_payload`  — coords ~ U[0,100]^2, D = round(euclid) (int, symmetric, 0 diagonal),
                       W[f,i] = Bernoulli(rho) * U{1..50}, workload_on_destination = 1,
                       cores_matrix ~ U(0.01, 0.1), cores ~ U{8..64}, node_mem ~ U{64..256},
                       fn_mem ~ U{4..32}, every function pre-allocated on 2 random nodes.
`alibaba_payload`    — the Alibaba-trace shape (`testing/alibaba/alibaba_test.py:374-400`):
                       node mem 100, cores 96, fn mem in {0.1,0.2,0.3,0.39,0.49},
                       no delay matrix (D = 1 - I), W == 0, ~0.6 % of (f,j) pre-allocated.
"""
import numpy as np


def _names(prefix, k, namespace=None):
    if namespace is None:
        return [f"{prefix}{i}" for i in range(k)]
    return [f"{namespace}/{prefix}{i}" for i in range(k)]


def synthetic_payload(n_nodes, n_functions, seed=0, rho=0.1, alpha=0.5,
                      solver_type="NeptuneMinDelayAndUtilization", soften_step1_sol=1.3,
                      prealloc_per_function=2):
    rng = np.random.default_rng(seed)
    N, F = int(n_nodes), int(n_functions)
    xy = rng.uniform(0.0, 100.0, size=(N, 2))
    diff = xy[:, None, :] - xy[None, :, :]
    D = np.rint(np.sqrt((diff ** 2).sum(-1))).astype(np.int64)
    D = np.minimum(D, D.T)
    np.fill_diagonal(D, 0)
    active = rng.random((F, N)) < rho
    W = np.where(active, rng.integers(1, 51, size=(F, N)), 0).astype(np.int64)
    cores_matrix = np.round(rng.uniform(0.01, 0.1, size=(F, N)), 4)
    cores = rng.integers(8, 65, size=N)
    node_mem = rng.integers(64, 257, size=N)
    fn_mem = rng.integers(4, 33, size=F)
    nodes = _names("node_", N)
    funcs = _names("fn_", F, "ns")
    alloc = {}
    k = min(prealloc_per_function, N)
    for f in range(F):
        js = rng.choice(N, size=k, replace=False)
        alloc[funcs[f]] = {nodes[j]: True for j in sorted(js.tolist())}
    return {
        "with_db": False,
        "solver": {"type": solver_type,
                   "args": {"alpha": alpha, "verbose": False, "soften_step1_sol": soften_step1_sol}},
        "workload_coeff": 1,
        "community": "community-synthetic",
        "namespace": "ns",
        "node_names": nodes,
        "node_memories": node_mem.tolist(),
        "node_cores": cores.tolist(),
        "gpu_node_names": [],
        "gpu_node_memories": [],
        "function_names": funcs,
        "function_memories": fn_mem.tolist(),
        "function_max_delays": [1000] * F,
        "gpu_function_names": [],
        "gpu_function_memories": [],
        "node_delay_matrix": D.tolist(),
        "workload_on_source_matrix": W.tolist(),
        "workload_on_destination_matrix": np.ones((F, N), np.int64).tolist(),
        "cores_matrix": cores_matrix.tolist(),
        "actual_cpu_allocations": alloc,
        "actual_gpu_allocations": {},
    }


def alibaba_payload(n_nodes=1024, n_functions=512, seed=0, alpha=0.5,
                    solver_type="NeptuneMinDelayAndUtilization", prealloc_frac=0.006):
    rng = np.random.default_rng(seed)
    N, F = int(n_nodes), int(n_functions)
    nodes = _names("m_", N)
    funcs = _names("task_", F, "j")
    mems = np.array([0.1, 0.2, 0.3, 0.39, 0.49])
    fn_mem = mems[rng.integers(0, len(mems), size=F)]
    n_alloc = max(1, int(round(prealloc_frac * F * N)))
    flat = rng.choice(F * N, size=n_alloc, replace=False)
    alloc = {}
    for idx in sorted(flat.tolist()):
        f, j = divmod(idx, N)
        alloc.setdefault(funcs[f], {})[nodes[j]] = True
    return {
        "with_db": False,
        "solver": {"type": solver_type, "args": {"alpha": alpha, "verbose": False}},
        "community": "community-trace",
        "namespace": "namespace-trace",
        "node_names": nodes,
        "node_memories": [100] * N,
        "node_cores": [96] * N,
        "gpu_node_names": [],
        "gpu_node_memories": [],
        "function_names": funcs,
        "function_memories": fn_mem.tolist(),
        "function_max_delays": [100] * F,
        "gpu_function_names": [],
        "gpu_function_memories": [],
        "actual_cpu_allocations": alloc,
        "actual_gpu_allocations": {},
    }
