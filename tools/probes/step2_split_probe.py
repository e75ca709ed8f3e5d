#!/usr/bin/env python3
"""Dev probe (GPU box): where an uncertified step-2 LP loses its certificate — the routing or the small
block.  Each LP is solved cold to BUDGET iterations; for every LP that does not certify, the routing
iterate x is fetched and the LP is re-solved by HiGHS over the small variables only (c, moved, a, d, n)
with x held fixed (rows over x alone are checked, not imposed; the score row gets the certificate's
relative tolerance).  Printed per LP: the engine's repaired-point objective (pobj), the best objective
any small block reaches at that x (best|x), HiGHS's LP value (ref) and the x-only row violations.  If
best|x is within tol of ref while pobj is not, the repaired point's small block is what fails.

  BUDGET=200000 python3 tools/step2_split_probe.py payload:1 scale:syn64x32_MDU_s2delete
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests"),
                os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
from scipy.optimize import Bounds, LinearConstraint, milp  # noqa: E402


def case(arg):
    """(data, variant, step, kw, oracle model, [(z_int lb, ub, ref)] root first)."""
    if arg.startswith("scale:"):
        from gen_scale_golden import model_of
        from scale_util import case_model_args, scale_cases
        c = scale_cases()[arg[6:]]
        data, variant, step, kw = case_model_args(c)
        mdl, _ = model_of(c)
        n_int = c["n_int"]
        lps = [(None, None, c["root"]["lp_objective"])]
        for nd in c["nodes"]:
            lb = np.full(n_int, -np.inf)
            ub = np.full(n_int, np.inf)
            lb[nd["fix_idx"]] = nd["fix_val"]
            ub[nd["fix_idx"]] = nd["fix_val"]
            lps.append((lb, ub, nd["lp_objective"]))
        return data, variant, step, kw, mdl, lps
    from golden_util import model
    from gpu_cases import G, build_args, fixing_bounds
    name, k = arg.split(":")
    data, variant, step, kw = build_args(name, int(k))
    mdl = model(name, int(k))
    N, F = len(data.nodes), len(data.functions)
    n_int = mdl["c"].shape[0] - N * N * F
    lps = [(None, None, G[name]["models"][int(k)]["lp_objective"])] + fixing_bounds(name, int(k), n_int, N * N * F)
    return data, variant, step, kw, mdl, lps


def best_small_block(mdl, nx, xv, lb_int, ub_int, tol):
    A = mdl["A"].tocsr()
    Ax, As = A[:, :nx], A[:, nx:]
    r = Ax @ xv
    lo, hi = mdl["lo"], mdl["hi"]
    nnz_s = np.diff(As.indptr)
    nnz_x = np.diff(Ax.indptr)
    xonly = nnz_s == 0
    rn = np.maximum(1.0, abs(A).max(axis=1).toarray().ravel())
    viol = np.maximum(np.maximum(lo - r, r - hi), 0.0) / rn
    mixed = ~xonly
    relax = np.where(mixed & (nnz_x > 0) & (nnz_x > np.sqrt(nx)), tol * rn, 0.0)
    lo_s = (lo - r - relax)[mixed]
    hi_s = (hi - r + relax)[mixed]
    lb = mdl["lb"][nx:].copy()
    ub = mdl["ub"][nx:].copy()
    if lb_int is not None:
        f = np.isfinite(lb_int)
        lb[f] = lb_int[f]
        ub[f] = ub_int[f]
    res = milp(mdl["c"][nx:], constraints=[LinearConstraint(As[mixed], lo_s, hi_s)],
               integrality=np.zeros(len(lb)), bounds=Bounds(lb, ub))
    val = None if res.x is None else float(mdl["c"][nx:] @ res.x + mdl["c"][:nx] @ xv)
    return val, float(viol[xonly].max()) if xonly.any() else 0.0, res.status


def repaired(mdl, data, step, nx, xv, zi, lb_int, ub_int, rule):
    """The certificate's repaired point on the host (fp64): rule 'A' = the T output clamped into
    [S/M, S + eps] (the engine's rule), 'B' = per column the c minimising the disruption cost given S
    (mf / mt / a / d at their cheapest; the price of sum c fixed by the mode).  Returns (objective,
    max relative row violation, row index of it)."""
    N, F = len(data.nodes), len(data.functions)
    FN = F * N
    lb = mdl["lb"][nx:].copy()
    ub = mdl["ub"][nx:].copy()
    if lb_int is not None:
        f = np.isfinite(lb_int)
        lb[f] = lb_int[f]
        ub[f] = ub_int[f]
    M, eps = 1e6, 1e-6
    S = xv.reshape(F, N, N).sum(axis=1).ravel()          # [f, j]
    old = np.asarray(data.old_allocations_matrix, np.float64).ravel()
    lo = np.maximum(lb[:FN], S / M)
    hi = np.minimum(ub[:FN], S + eps)
    cT = zi[:FN]
    cA = np.where(lo > hi, lo, np.minimum(np.maximum(cT, lo), hi))
    w = float(FN)
    sig4 = 1.0 if step == 3 else -1.0
    lam = -(w - 1) if step == 3 else (w + 1)
    if rule == "A":
        c = cA
    else:
        lmf, lmt = lb[FN:2 * FN], lb[2 * FN:3 * FN]
        cands = np.stack([lo, hi, np.clip(old + lmf, lo, hi), np.clip(old - lmt, lo, hi)])
        g = w * np.maximum(lmf, cands - old) + w * np.maximum(lmt, old - cands) + lam * cands
        c = np.where(lo > hi, lo, cands[np.argmin(g, axis=0), np.arange(FN)])
    z = np.zeros(len(lb))
    z[:FN] = c
    z[FN:2 * FN] = np.maximum(lb[FN:2 * FN], c - old)
    z[2 * FN:3 * FN] = np.maximum(lb[2 * FN:3 * FN], old - c)
    s = c.sum() - old.sum()
    ia, idd = 3 * FN, 3 * FN + 1
    A_ = min(ub[ia], -s)
    ar = max(lb[ia], A_)
    z[ia] = ar
    z[idd] = max(lb[idd], sig4 * (-s) - ar)
    if len(lb) > 3 * FN + 2:
        n0 = 3 * FN + 2
        sc = c.reshape(F, N).sum(axis=0)
        nlo = np.maximum(lb[n0:], sc / M)
        nhi = np.minimum(ub[n0:], sc + eps)
        nT = zi[n0:]
        z[n0:] = np.where(nlo > nhi, nlo, np.minimum(np.maximum(nT, nlo), nhi))
    full = np.concatenate([xv, z])
    r = mdl["A"] @ full
    rn = np.maximum(1.0, abs(mdl["A"]).max(axis=1).toarray().ravel())
    v = np.maximum(np.maximum(mdl["lo"] - r, r - mdl["hi"]), 0.0) / rn
    bv = np.maximum(np.maximum(lb - z, z - ub), 0.0)
    return float(mdl["c"] @ full), float(max(v.max(), bv.max())), int(np.argmax(v))


def main():
    from core.engine.lp import LPModel
    budget = int(os.environ.get("BUDGET", "200000"))
    ce = int(os.environ.get("CHECK_EVERY", "64"))
    tol = 5e-7
    for arg in sys.argv[1:]:
        data, variant, step, kw, mdl, lps = case(arg)
        N, F = len(data.nodes), len(data.functions)
        nx = N * N * F
        lps = lps[:int(os.environ.get("MAX_LPS", "9"))]
        B = len(lps)
        m = LPModel(data, variant, step=step, max_batch=B, **kw)
        lb = np.full((B, m.n_int), -np.inf)
        ub = np.full((B, m.n_int), np.inf)
        for b, (l, u, _) in enumerate(lps):
            if l is not None:
                lb[b], ub[b] = l, u
        res = m.solve(np.arange(B), lb, ub, tol=tol, max_iters=budget, check_every=ce)
        print(f"== {arg} (step {step}, {variant}, {N}x{F}) budget {budget}", flush=True)
        for b, (l, u, ref) in enumerate(lps):
            dg = m.diag(b)
            st = int(res["status"][b])
            line = (f"  lp {b}: st {st} it {int(res['iters'][b]):7d} ref {ref!s:>18} pobj-ref "
                    f"{(dg['pobj'] - ref) if ref is not None else float('nan'):+.3e} ref-bestL "
                    f"{(ref - dg['best_lagr']) if ref is not None else float('nan'):+.3e} res {dg['pres']:.2e}")
            if st != 0 and ref is not None:
                zi, x = m.solution(b)
                xv = x.astype(np.float64).transpose(1, 0, 2).ravel()     # [i][f][j] -> (f, i, j)
                val, xviol, hst = best_small_block(mdl, nx, xv, l, u, tol)
                line += (f" | best|x-ref {(val - ref) if val is not None else float('nan'):+.3e} (HiGHS st {hst})"
                         f" x-row viol {xviol:.2e}")
                if step >= 2:
                    for rule in ("A", "B"):
                        o, vv, vr = repaired(mdl, data, step, nx, xv, zi, l, u, rule)
                        line += f" | {rule}: obj-ref {o - ref:+.3e} viol {vv:.2e} (row {vr})"
            print(line, flush=True)
        m.close()


if __name__ == "__main__":
    main()
