#!/usr/bin/env python3
"""Dev probe (GPU box): why a node LP does not certify.  Solves golden LPs (tests/golden, as
tests/test_gpu_lp.py does), prints the engine's certificate diagnostics (nep_lp_get_diag: primal
objective of the repaired point, Lagrangian, max violation) and a host re-evaluation of the repaired
point from the engine's solution (routing rows + integer vector), row family by row family."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def host_repair(m, data, slot, lb, ub, step, kw):
    W = np.asarray(data.workload_matrix, float)
    F, N = W.shape
    xb, rf, rs = m.rows(slot)
    x = xb.astype(np.float64)
    zero = (W == 0).sum(axis=1).astype(float)
    wr = np.where(rs >= 0, 1.0, zero[rf])
    S = np.zeros((F, N))
    np.add.at(S, rf, wr[:, None] * x)
    z, _ = m.solution(slot, dense_x=False)
    L = m.layout()
    nat_lb = np.zeros(m.n_int)
    nat_ub = np.ones(m.n_int)
    if step != 1:
        nat_lb[L["allocated"][0]] = nat_lb[L["deallocated"][0]] = -F * N
        nat_ub[L["allocated"][0]] = nat_ub[L["deallocated"][0]] = 0
    blb = np.maximum(nat_lb, np.where(np.isfinite(lb), lb, -np.inf))
    bub = np.minimum(nat_ub, np.where(np.isfinite(ub), ub, np.inf))
    c0, c1 = L["c"]
    loc = np.maximum(blb[c0:c1].reshape(F, N), S / 1e6)
    hic = np.minimum(bub[c0:c1].reshape(F, N), S + 1e-6)
    out = {"C4": float(np.abs(x.sum(axis=1) - 1).max()), "c_empty": float((loc - hic).max()),
           "c_T_minus_rep": float(np.abs(z[c0:c1].reshape(F, N) - loc).max()),
           "rowsum_minmax": (float(x.sum(axis=1).min()), float(x.sum(axis=1).max()))}
    return out, S, z


def main():
    from core.engine.lp import LPModel
    from gpu_cases import G, build_args, fixing_bounds
    names = sys.argv[1:] or ["sim0_NeptuneMinDelay:1", "syn_8x4_s2_r0.1_NeptuneMinUtilization:0", "payload:0",
                             "sim3_NeptuneMinUtilization:1"]
    for nk in names:
        name, k = nk.split(":")
        k = int(k)
        data, variant, step, kw = build_args(name, k)
        rec = G[name]["models"][k]
        N, F = len(data.nodes), len(data.functions)
        nodes = fixing_bounds(name, k, 10 ** 9, N * N * F) if False else None
        m = LPModel(data, variant, step=step, max_batch=1 + len(rec.get("node_lps", [])), **kw)
        nodes = fixing_bounds(name, k, m.n_int, N * N * F)
        B = 1 + len(nodes)
        lb = np.full((B, m.n_int), -np.inf)
        ub = np.full((B, m.n_int), np.inf)
        for b, (l, u, _) in enumerate(nodes):
            lb[b + 1], ub[b + 1] = l, u
        for tol in (1e-7, 1e-6):
            res = m.solve(np.arange(B), lb, ub, tol=tol, max_iters=20000)
            refs = [rec["lp_objective"]] + [r for _, _, r in nodes]
            print(f"== {name} model {k} (step {step}, {variant}) tol {tol}", flush=True)
            for b in range(B):
                dg = m.diag(b)
                hr, _, _ = host_repair(m, data, b, lb[b], ub[b], step, kw)
                print(f"  node {b}: st {res['status'][b]} it {res['iters'][b]} obj {res['obj'][b]:.12g} "
                      f"ref {refs[b]} pobj_rep {dg['pobj']:.12g} lagr {dg['lagr']:.12g} res {dg['pres']:.3g} "
                      f"gap {dg['gap']:.3g} | host {hr}", flush=True)
        m.close()


if __name__ == "__main__":
    main()
