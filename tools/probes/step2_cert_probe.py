#!/usr/bin/env python3
"""Dev probe (GPU box): why a step-2 node LP does not certify — the repaired point's worst rows.  Solves the
golden LP (tests/gpu_cases: case, model, LP index) to the iteration limit and prints the engine's diagnostics,
then per (f, j): the column sum S (device flows), the repaired c / moved_from / moved_to, old, the node box,
and the C1/C2 (S vs c) and D1/D2 (moves vs c, old) violations; beside them HiGHS's optimum of the same LP.

  python3 tools/step2_cert_probe.py payload 1 1
  python3 tools/step2_cert_probe.py scale:syn64x32_MDU_s2delete 0 0     (tests/golden/scale.json cases)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def main():
    from core.engine.lp import LPModel
    from gpu_cases import build_args, fixing_bounds
    name, k, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    iters = int(os.environ.get("ITERS", "200000"))
    if name.startswith("scale:"):
        from scale_util import case_model_args, node_bounds, scale_cases
        c = scale_cases()[name[6:]]
        data, variant, step, kw = case_model_args(c)
        m = LPModel(data, variant, step=step, max_batch=2, **kw)
        lb = np.full((1, m.n_int), -np.inf)
        ub = np.full((1, m.n_int), np.inf)
        ref = c["root"].get("lp_objective")
        if b > 0:
            l, u = node_bounds(c, m.n_int)
            lb[0], ub[0] = l[b - 1], u[b - 1]
            ref = c["nodes"][b - 1].get("lp_objective")
    else:
        data, variant, step, kw = build_args(name, k)
        m = LPModel(data, variant, step=step, max_batch=2, **kw)
        ref = None
        lb = np.full((1, m.n_int), -np.inf)
        ub = np.full((1, m.n_int), np.inf)
    N, F = len(data.nodes), len(data.functions)
    nx = N * N * F
    if not name.startswith("scale:"):
        nodes = fixing_bounds(name, k, m.n_int, nx)
        if b > 0:
            l, u, ref = nodes[b - 1]
            lb[0], ub[0] = l, u
    r = m.solve([0], lb, ub, tol=5e-7, max_iters=iters)
    d = m.diag(0)
    print(f"{name} model {k} LP {b}: status {r['status'][0]} obj {r['obj'][0]:.10g} pobj {r['primal_obj'][0]:.10g} "
          f"HiGHS {ref} iters {r['iters'][0]} pres {d['pres']:.3e} gap {d['gap']:.3e} omega {d['omega']:.3g}", flush=True)
    z, _ = m.solution(0, dense_x=False)
    S = m.flows([0])[0].astype(np.float64)
    L = m.layout()
    c0, c1 = L["c"]
    c = z[c0:c1].reshape(F, N)
    old = np.asarray(data.old_allocations_matrix, np.float64).reshape(F, N)
    out = []
    mf = mt = None
    if "moved_from" in L:
        mf = z[L["moved_from"][0]:L["moved_from"][1]].reshape(F, N)
        mt = z[L["moved_to"][0]:L["moved_to"][1]].reshape(F, N)
    blb = lb[0][c0:c1].reshape(F, N)
    bub = ub[0][c0:c1].reshape(F, N)
    for f in range(F):
        for j in range(N):
            v1 = max(0.0, S[f, j] - 1e6 * c[f, j])
            v2 = max(0.0, c[f, j] - 1e-6 - S[f, j])
            vd1 = vd2 = 0.0
            if mf is not None:
                vd1 = max(0.0, -old[f, j] - (mf[f, j] - c[f, j]))   # D1: mf - c >= -old
                vd2 = max(0.0, old[f, j] - (mt[f, j] + c[f, j]))    # D2: mt + c >= old
            out.append((max(v1, v2, vd1, vd2), f, j, S[f, j], c[f, j], old[f, j],
                        None if mf is None else mf[f, j], None if mt is None else mt[f, j], blb[f, j], bub[f, j],
                        v1, v2, vd1, vd2))
    out.sort(key=lambda t: -t[0])
    print(f"  flow on placements with old = 0: {float(S[old == 0].sum()):.6g}; sum c {float(c.sum()):.6g}; "
          f"sum old {float(old.sum()):.6g}; sum mf {0 if mf is None else float(mf.sum()):.6g}; "
          f"sum mt {0 if mt is None else float(mt.sum()):.6g}")
    print("  worst (f, j): viol S c old mf mt box_lb box_ub | C1 C2 D1 D2")
    for t in out[:8]:
        print("   ", t[1:3], " ".join(f"{v:.7g}" if v is not None else "-" for v in t[3:10]), "|",
              " ".join(f"{v:.2e}" for v in t[10:]), flush=True)
    # the moved_from / moved_to boxes of the fixed ones
    if mf is not None:
        o0, o1 = L["moved_to"]
        fixed_mt = [(i // N, i % N, lb[0][o0 + i], ub[0][o0 + i]) for i in range(F * N) if np.isfinite(ub[0][o0 + i])]
        print("  moved_to boxes:", fixed_mt[:10])
    m.close()


if __name__ == "__main__":
    main()
