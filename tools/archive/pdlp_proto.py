#!/usr/bin/env python3
"""Dev-only numpy prototype of restarted (Halpern / averaged) PDHG on a generic CSR LP.

Used to pick the algorithm variant and measure iteration counts on NEPTUNE models before
the HIP kernels are written.  Not part of the product or of the oracle.

    l_r <= (A z)_r <= u_r,  lb <= z <= ub,  min c^T z
"""
import argparse
import numpy as np
import scipy.sparse as sp
from scipy.optimize import linprog


def load_npz(path):
    z = np.load(path)
    A = sp.csr_matrix((z["A_data"], z["A_indices"], z["A_indptr"]), shape=tuple(z["A_shape"]))
    return dict(A=A, lo=z["lo"], hi=z["hi"], c=z["c"], lb=z["lb"], ub=z["ub"], ref=float(z["lp_objective"]))


def ruiz_pc(A, iters=10, pc_alpha=1.0):
    m, n = A.shape
    dr = np.ones(m)
    dc = np.ones(n)
    K = A.copy().tocsr()
    for _ in range(iters):
        rmax = np.sqrt(abs(K).max(axis=1).toarray().ravel())
        cmax = np.sqrt(abs(K).max(axis=0).toarray().ravel())
        rmax[rmax == 0] = 1
        cmax[cmax == 0] = 1
        K = sp.diags(1 / rmax) @ K @ sp.diags(1 / cmax)
        dr /= rmax
        dc /= cmax
    if pc_alpha is not None:
        Ka = abs(K)
        rn = np.sqrt(np.asarray(Ka.power(2 - pc_alpha).sum(axis=1)).ravel() if False else np.asarray(Ka.sum(axis=1)).ravel())
        cn = np.sqrt(np.asarray(Ka.sum(axis=0)).ravel())
        rn[rn == 0] = 1
        cn[cn == 0] = 1
        K = sp.diags(1 / rn) @ K @ sp.diags(1 / cn)
        dr /= rn
        dc /= cn
    return K.tocsr(), dr, dc


def power_norm(K, iters=60, seed=0):
    v = np.random.default_rng(seed).standard_normal(K.shape[1])
    for _ in range(iters):
        v = K.T @ (K @ v)
        nv = np.linalg.norm(v)
        v /= nv
    return np.sqrt(nv)


def solve(m, tol=1e-6, max_iter=200000, halpern=True, reflect=1.0, verbose=False, check_every=64, scale=True):
    A, lo, hi, c, lb, ub = m["A"], m["lo"], m["hi"], m["c"], m["lb"], m["ub"]
    if scale:
        K, dr, dc = ruiz_pc(A)
    else:
        K, dr, dc = A.tocsr(), np.ones(A.shape[0]), np.ones(A.shape[1])
    # scaled problem in variables zt = z / dc ; rows scaled by dr
    cs = c * dc
    los, his = lo * dr, hi * dr
    lbs, ubs = lb / dc, ub / dc
    KT = K.T.tocsr()
    eta = 0.998 / power_norm(K)
    bnorm = np.linalg.norm(np.concatenate([np.where(np.isfinite(los), los, 0), np.where(np.isfinite(his), his, 0)]))
    cnorm = np.linalg.norm(cs)
    omega = cnorm / bnorm if (cnorm > 1e-10 and bnorm > 1e-10) else 1.0
    n, mm = K.shape[1], K.shape[0]
    z = np.clip(np.zeros(n), lbs, ubs)
    y = np.zeros(mm)
    z0, y0 = z.copy(), y.copy()
    k_since = 0
    total = 0
    last_restart_err = None
    prev_err = np.inf

    def T(z, y):
        tau, sig = eta / omega, eta * omega
        zn = np.clip(z - tau * (cs - KT @ y), lbs, ubs)
        v = y - sig * (K @ (2 * zn - z))
        yn = v - sig * np.clip(v / sig, -his, -los)
        return zn, yn

    def kkt(z, y):
        Kz = K @ z
        pres = Kz - np.clip(Kz, los, his)
        rc = cs - KT @ y
        # dual residual: rc must be >=0 where z at lb (finite), <=0 where at ub, 0 otherwise
        rc_l = np.where(np.isfinite(lbs), np.maximum(rc, 0), 0)
        rc_u = np.where(np.isfinite(ubs), np.minimum(rc, 0), 0)
        dres = rc - rc_l - rc_u
        pobj = cs @ z
        ypos = np.maximum(y, 0)
        yneg = np.minimum(y, 0)
        dobj = (np.where(np.isfinite(los), los, 0) @ ypos + np.where(np.isfinite(his), his, 0) @ yneg
                + np.where(np.isfinite(lbs), lbs, 0) @ rc_l + np.where(np.isfinite(ubs), ubs, 0) @ rc_u)
        pr = np.linalg.norm(pres / dr)
        du = np.linalg.norm(dres / dc)
        return pr, du, pobj, dobj

    hist = []
    while total < max_iter:
        zn, yn = T(z, y)
        if halpern:
            kk = k_since
            zr = (1 + reflect) * zn - reflect * z
            yr = (1 + reflect) * yn - reflect * y
            z_next = (kk + 1) / (kk + 2) * zr + 1 / (kk + 2) * z0
            y_next = (kk + 1) / (kk + 2) * yr + 1 / (kk + 2) * y0
        else:
            z_next, y_next = zn, yn
        total += 1
        k_since += 1
        if total % check_every == 0:
            pr, du, pobj, dobj = kkt(zn, yn)
            gap = abs(pobj - dobj)
            err = np.sqrt(pr ** 2 + du ** 2 + gap ** 2)
            ok = (pr <= tol * (1 + bnorm)) and (du <= tol * (1 + cnorm)) and gap <= tol * (1 + abs(pobj) + abs(dobj))
            hist.append((total, pr, du, pobj, dobj))
            if verbose:
                print(f"{total:7d} pr={pr:.2e} du={du:.2e} p={pobj:.9g} d={dobj:.9g} w={omega:.3g}")
            if ok:
                return zn * dc, yn * dr, total, pobj, dobj, hist
            # fixed-point residual based restart
            fpr = np.sqrt(omega * np.sum((zn - z) ** 2) + np.sum((yn - y) ** 2) / omega)
            if last_restart_err is None:
                last_restart_err = fpr
            do_restart = (fpr <= 0.2 * last_restart_err) or (fpr <= 0.8 * last_restart_err and fpr > prev_err) \
                or (k_since >= 0.36 * total)
            prev_err = fpr
            if do_restart:
                # primal weight update
                dz = np.linalg.norm(zn - z0)
                dy = np.linalg.norm(yn - y0)
                if dz > 1e-10 and dy > 1e-10:
                    omega = np.exp(0.5 * np.log(dy / dz) + 0.5 * np.log(omega))
                z0, y0 = zn.copy(), yn.copy()
                z_next, y_next = zn, yn
                k_since = 0
                last_restart_err = fpr
                prev_err = np.inf
        z, y = z_next, y_next
    pr, du, pobj, dobj = kkt(zn, yn)
    return zn * dc, yn * dr, total, pobj, dobj, hist


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--avg", action="store_true")
    ap.add_argument("-v", action="store_true")
    args = ap.parse_args()
    m = load_npz(args.npz)
    z, y, it, p, d, _ = solve(m, tol=args.tol, halpern=not args.avg, verbose=args.v)
    print(f"iters={it} pobj={m['c'] @ z:.10g} dobj={d:.10g} ref={m['ref']:.10g} gap={abs(m['c'] @ z - m['ref']):.2e}")
