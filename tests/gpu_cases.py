"""Shared helpers for the GPU parity tests: golden model -> product LPModel arguments."""
import numpy as np

from golden_util import golden, model, payload

VARIANT = {"NeptuneMinDelayAndUtilization": "MinDelayAndUtilization", "NeptuneMinDelay": "MinDelay",
           "NeptuneMinUtilization": "MinUtilization"}
G = golden()


def lp_cases(max_vars=5000):
    import os
    from golden_util import GOLDEN
    out = []
    for name, v in G.items():
        if "models" not in v:
            continue
        for k, m in enumerate(v["models"]):
            have = os.path.exists(os.path.join(GOLDEN, "models", f"{name}__0.npz"))
            if have and m["n_vars"] <= max_vars and m.get("lp_objective") is not None:
                out.append((name, k))
    return out


def build_args(name, k):
    """(data, variant, step, kwargs) for the k-th recorded model of a golden case."""
    from core.utils import data_to_solver_input
    p = payload(name)
    data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
    variant = VARIANT[p["solver"]["type"]]
    args = p["solver"].get("args", {})
    kw = dict(alpha=args.get("alpha", 0.5), soften_step1_sol=args.get("soften_step1_sol", 1.3))
    if k == 0:
        return data, variant, 1, kw
    m1 = model(name, 0)
    N, F = len(data.nodes), len(data.functions)
    kw["max_score"] = float(m1["mip_objective"])
    x1 = m1["mip_x"][:N * N * F].reshape(F, N, N)       # [f,i,j]
    D = data.node_delay_matrix.astype(np.float64)
    W = data.workload_matrix.astype(np.float64)
    kw["prev_network_delay"] = float(np.sum(D[None, :, :] * W[:, :, None] * x1))
    return data, variant, 1 + k, kw


def fixing_bounds(name, k, n_int, nx):
    """Golden node fixings (indices into the reference variable vector) -> z_int bounds."""
    out = []
    for nl in G[name]["models"][k].get("node_lps", []):
        lb = np.full(n_int, -np.inf)
        ub = np.full(n_int, np.inf)
        for i, val in zip(nl["fix_idx"], nl["fix_val"]):
            lb[i - nx] = val
            ub[i - nx] = val
        out.append((lb, ub, nl["lp_objective"]))
    return out
