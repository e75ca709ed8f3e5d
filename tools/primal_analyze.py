#!/usr/bin/env python3
"""Dev analysis (CPU) of tools/primal_probe.py dumps: rebuilds the certificate's repaired primal point
 from the engine's routing rows and small-variable iterate, splits its objective into the
step-2 terms and compares them, pair by pair, with the HiGHS optimum of the same LP (oracle).

  python3 tools/primal_analyze.py gpurun_out/r03d/primal_scale_syn64x32_MDU_s2delete.npz scale:syn64x32_MDU_s2delete
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402


def main():
    d = np.load(sys.argv[1])
    arg = sys.argv[2]
    from step2_probe import case
    from gen_scale_golden import model_of, cases
    from oracle.solve import solve
    data, variant, step, kw, rootref, nodes, scale = case(arg)
    F, N = data.workload_matrix.shape
    FN = F * N
    M, eps = 1e6, 1e-6
    W = np.asarray(data.workload_matrix, float)
    xb, rf, rs, z = d["xb"].astype(np.float64), d["rf"], d["rs"], d["z"]
    m = np.where(rs >= 0, 1.0, (W == 0).sum(axis=1)[rf])
    S = np.zeros((F, N))
    np.add.at(S, rf, m[:, None] * xb)
    S = S.ravel()
    old = np.asarray(data.old_allocations_matrix, float).ravel()
    c_it = z[:FN]
    c = np.clip(c_it, S / M, S + eps)
    mf, mt = np.maximum(0, c - old), np.maximum(0, old - c)
    w = float(FN)
    sig4 = 1.0 if step == 3 else -1.0
    s = c.sum() - old.sum()
    A, Dm, K = min(0.0, -s), min(0.0, s), sig4 * (-s)
    ar = max(-FN, A)
    dr = max(-FN, K - ar)
    pobj = w * (mf.sum() + mt.sum()) + (w - 1) * ar + (w + 1) * dr
    print(f"engine pobj {float(d['pobj']):.10g}  rebuilt {pobj:.10g}  ref {float(d['ref']):.10g}  bestL {float(d['bestl']):.10g}")
    print(f"  w sum mf {w * mf.sum():.6g}  w sum mt {w * mt.sum():.6g}  (w-1) a {(w - 1) * ar:.6g}  (w+1) d {(w + 1) * dr:.6g}"
          f"  sum c - sum old {s:.6g}")
    # HiGHS
    c0 = [c for c in cases() if c["name"] == arg.split(":")[1]][0] if scale else None
    if c0 is not None:
        mo, dd = model_of(c0)
        st, obj, x = solve(mo, relax=True)
        nx = N * N * F
        X = x[:nx].reshape(F, N, N)
        Sh = X.sum(axis=1).ravel()
        ch = x[nx:nx + FN]
        mfh, mth = x[nx + FN:nx + 2 * FN], x[nx + 2 * FN:nx + 3 * FN]
        print(f"HiGHS obj {obj:.10g}: w sum mf {w * mfh.sum():.6g} w sum mt {w * mth.sum():.6g} a {x[nx + 3 * FN]:.6g} "
              f"d {x[nx + 3 * FN + 1]:.6g} sum c - sum old {ch.sum() - old.sum():.6g}")
        dc = c - ch
        order = np.argsort(-np.abs(dc))[:12]
        print("largest |c_rep - c_highs| pairs (f, j, old, c_it, c_rep, c_highs, S, S_highs):")
        for k in order:
            print(f"  {k // N:4d} {k % N:4d} {old[k]:.0f} {c_it[k]:.9f} {c[k]:.9f} {ch[k]:.9f} {S[k]:.9f} {Sh[k]:.9f}")
        print("pairs with c_rep != c_highs beyond 1e-9:", int((np.abs(dc) > 1e-9).sum()),
              " sum (c_rep - c_highs):", float(dc.sum()))


if __name__ == "__main__":
    main()
