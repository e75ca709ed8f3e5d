#!/usr/bin/env python3
"""Dev-only: algorithm variants of the engine's PDHG on the numpy mirror (tests/ref_pdhg.py) —
currently reflected restarted Halpern PDHG (Lu & Yang, r2HPDHG) against the plain restarted PDHG
the kernels run.  Usage: pdhg_variants.py N F {plain|halpern} [max_iters] [rho]"""
import sys
import time

sys.path[:0] = ["/root/repo/neptune-mip_amd", "/root/repo", "/root/repo/tests"]
import numpy as np  # noqa: E402
import ref_pdhg  # noqa: E402
from ref_pdhg import INF, proj_simplex_rows  # noqa: E402


def lagrangian(m, y, cost_x, mask, lb, ub):
    gx, gz = m.KT(y)
    rcx = cost_x - gx
    rcz = m.cost_int - gz
    lag = np.where(mask, rcx, INF).min(axis=1).sum()
    lag += np.where(rcz > 0, lb * rcz, ub * rcz).sum()
    with np.errstate(invalid="ignore"):
        rl = np.where(y > 0, np.where(np.isfinite(m.lo), y * m.lo, -INF),
                      np.where(y < 0, np.where(np.isfinite(m.hi), y * m.hi, -INF), 0.0))
    return lag + rl.sum()


def solve(m, lbi=None, ubi=None, tol=1e-6, max_iters=100000, check_every=64, halpern=True, reflect=True,
          verbose=False):
    ok, lb, ub, fmask = m.presolve(lbi, ubi)
    mask = fmask[m.row_f]
    x = proj_simplex_rows(np.zeros((m.R, m.N)), mask)
    z = np.clip(np.zeros(m.n_int), lb, ub)
    y = np.zeros(m.n_dual)
    kz = m.K(x, z)
    xa, za, ya, kza = x.copy(), z.copy(), y.copy(), kz.copy()
    omega, eta = m.omega0, m.eta
    om_lo, om_hi = m.omega0 * 1e-5, m.omega0 * 1e5
    k = ks = 0
    last_fpr, prev_fpr = -1.0, INF
    best = -INF
    cost_x = m.row_wobj[:, None] * np.where(m.row_src[:, None] >= 0, m.D32[np.maximum(m.row_src, 0)], 0.0)
    while True:
        for it in range(check_every):
            tau, sig = eta / omega, eta * omega
            gx, gz = m.KT(y)
            xn = proj_simplex_rows(x - tau * (cost_x - gx), mask)
            zn = np.clip(z - tau * m.gam ** 2 * (m.cost_int - gz), lb, ub)
            act = m.K(xn, zn)
            s = sig * m.rho ** 2
            V = y - s * (2 * act - kz)
            with np.errstate(invalid="ignore"):
                a = V + s * m.hi
                b = V + s * m.lo
            yn = np.where(a < 0, a, np.where(b > 0, b, 0.0))
            if it == check_every - 1:
                lag = lagrangian(m, yn, cost_x, mask, lb, ub)
                pobj = (cost_x * xn).sum() + (m.cost_int * zn).sum()
                res = (np.maximum(np.maximum(m.lo - act, act - m.hi), 0.0) / m.rownorm).max()
                fx = ((xn - x) ** 2).sum() + (((zn - z) / m.gam) ** 2).sum()
                fy = (((yn - y) / m.rho) ** 2).sum()
                dsz = ((xn - xa) ** 2).sum() + (((zn - za) / m.gam) ** 2).sum()
                dsy = (((yn - ya) / m.rho) ** 2).sum()
                xT, zT, yT, kT = xn, zn, yn, act
            if halpern:
                lam = (ks + 1.0) / (ks + 2.0)
                r = 2.0 if reflect else 1.0
                x = lam * (r * xn - (r - 1) * x) + (1 - lam) * xa
                z = lam * (r * zn - (r - 1) * z) + (1 - lam) * za
                y = lam * (r * yn - (r - 1) * y) + (1 - lam) * ya
                kz = lam * (r * act - (r - 1) * kz) + (1 - lam) * kza
            else:
                x, z, y, kz = xn, zn, yn, act
            ks += 1
        k += check_every
        best = max(best, lag)
        gap = pobj - lag
        if verbose:
            print(f"{k:7d} res={res:.2e} p={pobj:.10g} L={lag:.10g} gap={gap:.2e} w={omega:.3g}", flush=True)
        if np.isfinite(lag) and res <= tol and gap <= tol * max(1.0, abs(lag)):
            return dict(status=0, obj=lag, pobj=pobj, iters=k)
        if k >= max_iters:
            return dict(status=1, obj=best, pobj=pobj, iters=k)
        fpr = np.sqrt(omega * fx + fy / omega)
        if last_fpr < 0:
            last_fpr = fpr
        restart = fpr <= 0.2 * last_fpr or (fpr <= 0.8 * last_fpr and fpr > prev_fpr) or ks >= 0.36 * k
        prev_fpr = fpr
        if restart:
            dz, dy = np.sqrt(dsz), np.sqrt(dsy)
            if dz > 1e-10 and dy > 1e-10:
                omega = float(np.clip(np.exp(0.5 * np.log(dy / dz) + 0.5 * np.log(omega)), om_lo, om_hi))
            x, z, y, kz = xT, zT, yT, kT          # restart at the PDHG output T(z)
            xa, za, ya, kza = x.copy(), z.copy(), y.copy(), kz.copy()
            ks = 0
            last_fpr = fpr
            prev_fpr = INF


if __name__ == "__main__":
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F, mode = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    mi = int(sys.argv[4]) if len(sys.argv) > 4 else 30000
    rho = float(sys.argv[5]) if len(sys.argv) > 5 else 0.1
    p = synthetic_payload(N, F, seed=0, rho=rho)
    d = data_to_solver_input(p, with_db=False)
    m = ref_pdhg.RefModel(d, "MinDelayAndUtilization", 1, alpha=0.5)
    t = time.time()
    r = solve(m, tol=1e-6, max_iters=mi, halpern=mode != "plain", reflect=mode != "halpern1", verbose=True)
    print(mode, "status", r["status"], "obj", r["obj"], "iters", r["iters"], f"{time.time() - t:.0f}s")
