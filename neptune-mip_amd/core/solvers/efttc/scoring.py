"""Host scorers and the two feasibility checks EF-TTC step 1 consults while it places functions
(reference `core/solvers/efttc/utils/objectives.py:23-98`, `utils/constraints_step1.py:57-133`),
on the numpy state of `efttc_step1.py`.  Same arithmetic (same numpy expressions, same
truthiness) so scores compare equal to the reference's.

The scorers/checkers of a solved NEPTUNE node run on the device instead
(`nep_lp_score_check`, csrc/nep_aux.hip; `LPModel.score_check`).
"""
import numpy as np


def network_delay(data, x):
    """score_minimize_network_delay (objectives.py:23-36): sum x[i,f,j] D[i,j] W[f,i]."""
    w = np.transpose(data.workload_matrix, (1, 0))[:, :, np.newaxis]
    d = data.node_delay_matrix[:, np.newaxis, :]
    return np.sum(np.asarray(x, np.float64) * d * w)


def node_utilization(data, n):
    """score_minimize_node_utilization (objectives.py:48-49): number of nodes with n set."""
    return sum(1 for j in range(len(data.nodes)) if n[j])


def node_delay_and_utilization(data, n, x, alpha):
    """score_minimize_node_delay_and_utilization (objectives.py:53-98)."""
    N, F = len(data.nodes), len(data.functions)
    util = sum(1 for j in range(N) if n[j]) * (alpha / N)
    W, D, md = data.workload_matrix, data.node_delay_matrix, data.max_delay_matrix
    if np.sum(W) == 0:
        return util
    dexp = np.broadcast_to(D, (F, N, N))
    masked = np.where(dexp <= md[:, np.newaxis, np.newaxis], dexp, 0)
    mwd = np.sum(W * masked.max(axis=2))
    if mwd == 0:
        return util
    xm = np.asarray(x, np.float32)
    contrib = xm * np.transpose(W, (1, 0))[:, :, np.newaxis] * D[:, np.newaxis, :]
    return util + np.sum(contrib) * (1 - alpha) / mwd


def cpu_usage_ok(data, x):
    """constrain_CPU_usage (constraints_step1.py:68-78): per node, sum_{f,i} x W cpr <= cores + 1e-6."""
    W, cpr, cores = data.workload_matrix, data.core_per_req_matrix, data.node_cores_matrix
    N, F = len(data.nodes), len(data.functions)
    lim = cores + 1e-6
    # vectorised totals decide every node not within rounding distance of its limit; those few are
    # re-summed in the reference's exact order (f outer, i inner) so the decision is bit-identical
    fast = np.einsum("ifj,fi,fj->j", x, W, cpr)
    close = np.abs(fast - lim) <= 1e-9 * np.maximum(1.0, np.abs(lim))
    if np.any((fast > lim) & ~close):
        return False
    for j in np.flatnonzero(close):
        total = 0
        for f in range(F):
            for i in range(N):
                total += x[i, f, j] * W[f, i] * cpr[f, j]
        if total > lim[j]:
            return False
    return True


def budget_ok(data, n):
    """constrain_budget (constraints_step1.py:127-133): sum n[j] cost[j] <= budget + 1e-6."""
    total = sum(n[j] * data.node_costs[j] for j in range(len(data.nodes)))
    return not (total > data.node_budget + 1e-6)
