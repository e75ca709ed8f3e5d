"""Test-only numpy mirror of the MI355X LP engine (neptune-mip_amd/csrc): same structured model
(zero-workload aggregation, coefficients, Ruiz + Pock-Chambolle scaling, power-iteration step) and
the same preconditioned PDHG iteration, restarts and certificate.  Used to (a) check the C++ model
build through nep_debug_build on CPU, (b) debug the algorithm without a GPU, (c) compare kernel
iterates.  Never used by the product path.
"""
import numpy as np

INF = np.inf


class RefModel:
    def __init__(self, data, variant, step=1, alpha=0.5, soften_step1_sol=1.3, max_score=0.0,
                 prev_network_delay=0.0, M=1e6, eps=1e-6, dred=None):
        D = np.asarray(data.node_delay_matrix, float)
        W = np.asarray(data.workload_matrix, float)
        F, N = W.shape
        cpr = np.asarray(data.core_per_req_matrix, float)
        cpr = np.where(np.isfinite(cpr), cpr, np.finfo(np.float32).max)
        self.N, self.F, self.M, self.eps = N, F, M, eps
        self.variant = {"MinDelay": 0, "MinUtilization": 1, "MinDelayAndUtilization": 2}.get(variant, variant)
        self.step2 = step != 1
        self.has_n = self.variant != 0
        self.sigma4 = 1.0 if step == 3 else -1.0
        rows = []
        for f in range(F):
            zeros = 0
            for i in range(N):
                if W[f, i] != 0:
                    rows.append((f, i, 1.0, W[f, i]))
                else:
                    zeros += 1
            if zeros:
                rows.append((f, -1, float(zeros), 0.0))
        self.R = len(rows)
        self.row_f = np.array([r[0] for r in rows])
        self.row_src = np.array([r[1] for r in rows])
        self.row_m = np.array([r[2] for r in rows], np.float32).astype(float)
        self.row_w = np.array([r[3] for r in rows], np.float32).astype(float)
        kobj = 0.0
        if not self.step2:
            if self.variant == 0:
                kobj = 1.0
            elif self.variant == 2 and W.sum() != 0:
                md = np.asarray(data.max_delay_matrix, float)
                mwd = 0.0
                for f in range(F):
                    for i in range(N):
                        mwd += W[f, i] * max(d for d in D[i] if d <= md[f])
                kobj = (1 - alpha) / mwd
            self.cost_n = {1: 1.0, 2: alpha / N}.get(self.variant, 0.0)
        else:
            self.cost_n = 0.0
        self.row_wobj = (kobj * self.row_w).astype(np.float32).astype(float)
        colmaxD = D.max(axis=0)
        wsc = np.zeros(self.R)
        self.score_n_coef = 0.0
        score_rhs = INF
        if self.step2:
            md = np.asarray(data.max_delay_matrix, float)
            for r in range(self.R):
                if self.row_src[r] >= 0:
                    if self.variant == 0:
                        wsc[r] = self.row_w[r]
                    elif self.variant == 2:
                        wsc[r] = (1 - alpha) * self.row_w[r] / max(md[self.row_f[r]], colmaxD[self.row_src[r]])
            if self.variant == 0:
                score_rhs = soften_step1_sol * prev_network_delay
            else:
                score_rhs = max_score * soften_step1_sol
                self.score_n_coef = 1.0 if self.variant == 1 else alpha / N
        self.row_wsc = wsc.astype(np.float32).astype(float)
        self.D32 = D.astype(np.float32).astype(float)
        self.cpr32 = cpr.astype(np.float32).astype(float)
        FN = F * N
        # int layout
        if not self.step2:
            self.oc, self.on = 0, (FN if self.has_n else -1)
            self.n_int = FN + (N if self.has_n else 0)
        else:
            self.oc, self.omf, self.omt, self.oa, self.od = 0, FN, 2 * FN, 3 * FN, 3 * FN + 1
            self.on = 3 * FN + 2 if self.has_n else -1
            self.n_int = 3 * FN + 2 + (N if self.has_n else 0)
        self.nat_lb = np.zeros(self.n_int)
        self.nat_ub = np.ones(self.n_int)
        self.cost_int = np.zeros(self.n_int)
        if self.has_n:
            cost = np.asarray(data.node_costs, float)
            for j in range(N):
                if cost[j] > 0:
                    self.nat_ub[self.on + j] = min(1.0, data.node_budget / cost[j])
                self.cost_int[self.on + j] = self.cost_n
        old = np.asarray(data.old_allocations_matrix, float).ravel()
        sum_old = old.sum()
        if self.step2:
            w = float(FN)
            self.cost_int[self.omf:self.omf + FN] = w
            self.cost_int[self.omt:self.omt + FN] = w
            self.cost_int[self.oa] = w - 1
            self.cost_int[self.od] = w + 1
            self.nat_lb[self.oa] = self.nat_lb[self.od] = -float(FN)
            self.nat_ub[self.oa] = self.nat_ub[self.od] = 0.0
        # dual layout
        o = 0
        self.o1 = o; o += FN
        self.o2 = o; o += FN
        self.o3 = o; o += N
        self.o5 = o; o += N
        if self.has_n:
            self.o6 = o; o += N
            self.o7 = o; o += N
        if self.step2:
            self.oD1 = o; o += FN
            self.oD2 = o; o += FN
            self.oD3a, self.oD3b, self.oD4, self.oS = o, o + 1, o + 2, o + 3
            o += 4
        self.n_dual = o
        lo = np.full(o, -INF)
        hi = np.full(o, INF)
        hi[self.o1:self.o1 + FN] = 0.0
        lo[self.o2:self.o2 + FN] = -eps
        hi[self.o3:self.o3 + N] = np.asarray(data.node_memory_matrix, float)
        hi[self.o5:self.o5 + N] = np.asarray(data.node_cores_matrix, float)
        if self.has_n:
            hi[self.o6:self.o6 + N] = 0.0
            lo[self.o7:self.o7 + N] = -eps
        if self.step2:
            lo[self.oD1:self.oD1 + FN] = -old
            lo[self.oD2:self.oD2 + FN] = old
            lo[self.oD3a] = -sum_old
            lo[self.oD3b] = sum_old
            lo[self.oD4] = self.sigma4 * sum_old
            hi[self.oS] = score_rhs
        self.lo, self.hi = lo, hi
        self.mem_f = np.asarray(data.function_memory_matrix, float)
        # COO of the non-x part
        r, c, v = [], [], []

        def add(a, b, val):
            r.append(a); c.append(b); v.append(val)
        for f in range(F):
            for j in range(N):
                k = f * N + j
                add(self.o1 + k, self.oc + k, -M)
                add(self.o2 + k, self.oc + k, -1.0)
                add(self.o3 + j, self.oc + k, self.mem_f[f])
                if self.has_n:
                    add(self.o6 + j, self.oc + k, 1.0)
                    add(self.o7 + j, self.oc + k, 1.0)
                if self.step2:
                    add(self.oD1 + k, self.omf + k, 1.0)
                    add(self.oD1 + k, self.oc + k, -1.0)
                    add(self.oD2 + k, self.omt + k, 1.0)
                    add(self.oD2 + k, self.oc + k, 1.0)
                    add(self.oD3a, self.oc + k, -1.0)
                    add(self.oD3b, self.oc + k, 1.0)
                    add(self.oD4, self.oc + k, self.sigma4)
        if self.has_n:
            for j in range(N):
                add(self.o6 + j, self.on + j, -M)
                add(self.o7 + j, self.on + j, -1.0)
                if self.step2 and self.score_n_coef != 0:
                    add(self.oS, self.on + j, self.score_n_coef)
        if self.step2:
            add(self.oD3a, self.oa, -1.0)
            add(self.oD3b, self.od, -1.0)
            add(self.oD4, self.od, 1.0)
            add(self.oD4, self.oa, 1.0)
        self.Kr, self.Kc, self.Kv = np.array(r), np.array(c), np.array(v)
        # x-row norms
        xmax = np.zeros(o)
        xsum = np.zeros(o)
        for f in range(F):
            sel = self.row_f == f
            mm, ms = (self.row_m[sel].max(), self.row_m[sel].sum()) if sel.any() else (0.0, 0.0)
            xmax[self.o1 + f * N:self.o1 + (f + 1) * N] = mm
            xmax[self.o2 + f * N:self.o2 + (f + 1) * N] = mm
            xsum[self.o1 + f * N:self.o1 + (f + 1) * N] = ms
            xsum[self.o2 + f * N:self.o2 + (f + 1) * N] = ms
        wc = self.row_w[:, None] * cpr[self.row_f]            # [R, N]
        xmax[self.o5:self.o5 + N] = np.abs(wc).max(axis=0)
        xsum[self.o5:self.o5 + N] = np.abs(wc).sum(axis=0)
        if self.step2:
            sc = self._score_coef(D)
            xmax[self.oS] = np.abs(sc).max() if sc.size else 0.0
            xsum[self.oS] = np.abs(sc).sum()
        self.wc = wc
        rn = np.maximum(1.0, xmax)
        rn = np.where(np.isfinite(lo), np.maximum(rn, np.abs(np.where(np.isfinite(lo), lo, 0))), rn)
        rn = np.where(np.isfinite(hi), np.maximum(rn, np.abs(np.where(np.isfinite(hi), hi, 0))), rn)
        np.maximum.at(rn, self.Kr, np.abs(self.Kv))
        self.rownorm = rn
        # step 2, reduced disruption block (nep_host.cpp build): mf / mt / a / d follow from c, the
        # iteration runs on K without D1/D2/D3a/D3b and with D4 as the row sum c (coefficient 1 on every c)
        self.old = old
        self.dred = bool(self.step2 and np.isin(old, (0.0, 1.0)).all()) if dred is None else bool(dred and self.step2)
        self.sT = 0.0
        if self.dred:
            self.sT = -(w - 1) if self.sigma4 > 0 else (w + 1)
            idle = np.zeros(o, bool)
            idle[self.oD1:self.oD1 + FN] = idle[self.oD2:self.oD2 + FN] = True
            idle[[self.oD3a, self.oD3b]] = True
            keep = ~idle[self.Kr]
            keep &= ~((self.Kr == self.oD4) & ((self.Kc < self.oc) | (self.Kc >= self.oc + FN)))
            self.Kr, self.Kc, self.Kv = self.Kr[keep], self.Kc[keep], self.Kv[keep]
            self.Kv = np.where(self.Kr == self.oD4, 1.0, self.Kv)
            lo[idle] = -INF
            hi[idle] = INF
        rho = np.ones(o)
        gam = np.ones(self.n_int)
        for sweep in range(11):
            pc = sweep == 10
            a = np.abs(rho[self.Kr] * self.Kv * gam[self.Kc])
            if pc:
                rnn = rho * xsum
                np.add.at(rnn, self.Kr, a)
                cn = np.zeros(self.n_int)
                np.add.at(cn, self.Kc, a)
            else:
                rnn = rho * xmax
                np.maximum.at(rnn, self.Kr, a)
                cn = np.zeros(self.n_int)
                np.maximum.at(cn, self.Kc, a)
            rho = np.where(rnn > 0, rho / np.sqrt(np.where(rnn > 0, rnn, 1)), rho)
            gam = np.where(cn > 0, gam / np.sqrt(np.where(cn > 0, cn, 1)), gam)
        self.rho, self.gam = rho, gam
        self.sigma_max = self._power()
        self.eta = 0.95 / self.sigma_max
        # initial primal weight ||c~|| / ||b~|| (scaled space), as nep_host.cpp build()
        cx = self.row_wobj[:, None] * np.where(self.row_src[:, None] >= 0, D[np.maximum(self.row_src, 0)], 0.0)
        # (reduced step 2: the reduced LP's costs and row bounds at natural bounds, as nep_host.cpp build)
        ci = self.cost_int
        if self.dred:
            ci, _, self.lo[self.oD4], self.hi[self.oD4] = self.dred_terms(self.nat_lb, self.nat_ub)
        cn2 = (self.row_m[:, None] * cx * cx).sum() + ((gam * ci) ** 2).sum()
        bmag = np.maximum(np.where(np.isfinite(lo), np.abs(lo), 0.0), np.where(np.isfinite(hi), np.abs(hi), 0.0))
        bn2 = ((rho * bmag) ** 2).sum()
        self.omega0 = float(np.sqrt(cn2) / np.sqrt(bn2)) if cn2 > 0 and bn2 > 0 else 1.0

    def dred_terms(self, lb, ub):
        """Reduced step 2 at a box: the iteration's costs (c: its own linear cost, mf / mt / a / d: 0), the
        objective's constant and the row sum c's bounds [L, U] (nep_device.h dred_cost / dred_bounds)."""
        FN, w = self.F * self.N, float(self.F * self.N)
        lmf, lmt = lb[self.omf:self.omf + FN], lb[self.omt:self.omt + FN]
        old0 = self.old < 0.5
        cost = self.cost_int.copy()
        cost[self.omf:self.omt + FN] = 0.0
        cost[self.oa] = cost[self.od] = 0.0
        cost[self.oc:self.oc + FN] = np.where(old0, np.where(lmf < 0.5, w, 0.0), np.where(lmt < 0.5, -w, 0.0)) + self.sT
        const = float(np.where(old0, w * (lmf + lmt), w * (lmf + 1.0)).sum()) - self.sT * self.old.sum()
        la, ua, ld, ud = lb[self.oa], ub[self.oa], lb[self.od], ub[self.od]
        if self.sigma4 > 0:
            ok = ld <= 0 <= ud
            tlo, thi = (max(0.0, -ua), -la) if ok else (1.0, 0.0)
        else:
            ok = la <= 0 <= ua
            tlo, thi = (ld, min(0.0, ud)) if ok else (1.0, 0.0)
        so = self.old.sum()
        return cost, const, so + tlo, so + thi

    def _score_coef(self, D):
        out = np.zeros((self.R, self.N))
        for r in range(self.R):
            if self.row_src[r] >= 0 and self.row_wsc[r] != 0:
                out[r] = self.row_wsc[r] * D[self.row_src[r]]
        return out

    # K·[x, z] (unscaled) and Kᵀy (unscaled)
    def K(self, x, z):
        N, F = self.N, self.F
        y = np.zeros(self.n_dual)
        S = np.zeros((F, N))
        np.add.at(S, self.row_f, self.row_m[:, None] * x)
        y[self.o1:self.o1 + F * N] += S.ravel()
        y[self.o2:self.o2 + F * N] += S.ravel()
        y[self.o5:self.o5 + N] += (self.wc * x).sum(axis=0)
        if self.step2:
            y[self.oS] += (self._score_coef(self.D32) * x).sum()
        np.add.at(y, self.Kr, self.Kv * z[self.Kc])
        return y

    def KT(self, y):
        N, F = self.N, self.F
        y12 = (y[self.o1:self.o1 + F * N] + y[self.o2:self.o2 + F * N]).reshape(F, N)
        gx = self.row_m[:, None] * y12[self.row_f] + self.wc * y[self.o5:self.o5 + N][None, :]
        if self.step2:
            gx = gx + self._score_coef(self.D32) * y[self.oS]
        gz = np.zeros(self.n_int)
        np.add.at(gz, self.Kc, self.Kv * y[self.Kr])
        return gx, gz

    def _power(self, iters=60):
        rng = np.random.default_rng(1)
        x = rng.standard_normal((self.R, self.N))
        z = rng.standard_normal(self.n_int)
        lam = 0.0
        for _ in range(iters):
            nrm = np.sqrt((x * x).sum() + (z * z).sum())
            x, z = x / nrm, z / nrm
            y = self.rho * self.K(x, self.gam * z)
            gx, gz = self.KT(self.rho * y)
            gz = gz * self.gam
            lam = (x * gx).sum() + (z * gz).sum()
            x, z = gx, gz
        return np.sqrt(max(lam, 1e-30))

    def presolve(self, lbi=None, ubi=None):
        lb = self.nat_lb.copy() if lbi is None else np.maximum(self.nat_lb, lbi)
        ub = self.nat_ub.copy() if ubi is None else np.minimum(self.nat_ub, ubi)
        N, F = self.N, self.F
        if self.has_n:
            for j in range(N):
                if ub[self.on + j] <= 0:
                    for f in range(F):
                        ub[self.oc + f * N + j] = min(ub[self.oc + f * N + j], 0.0)
        ok = not np.any(lb > ub + 1e-12)
        mask = (ub[self.oc:self.oc + F * N] > 0).reshape(F, N)
        if not mask.any(axis=1).all():
            ok = False
        return ok, lb, ub, mask


def proj_simplex_rows(V, mask):
    out = np.zeros_like(V)
    for r in range(V.shape[0]):
        v = V[r][mask[r]]
        if v.size == 0:
            continue
        u = np.sort(v)[::-1]
        css = np.cumsum(u)
        k = np.arange(1, len(u) + 1)
        rho = np.nonzero(u - (css - 1) / k > 0)[0][-1]
        theta = (css[rho] - 1) / (rho + 1)
        out[r][mask[r]] = np.maximum(v - theta, 0)
    return out


def solve(m, lbi=None, ubi=None, tol=1e-7, max_iters=100000, check_every=64, verbose=False, inline_reflect=False):
    """Same algorithm as the kernels, fp64: blocks of `check_every` iterations; iteration 0 of a block
    is the certificate iteration (a plain PDHG step whose input dual is the previous block's plain
    output), restarts take effect at iteration 1, the last iteration is plain, the others are
    reflected Halpern steps w' = lam (2 T(w) - w) + (1 - lam) w_anchor.
    inline_reflect: form the dual step's reflected activity as K(2ŵ - w) from the primal points
    (what x_pass does for the per-(f, j) rows) instead of 2·Kŵ - kz with the tracked activity kz;
    the two are the same operator (K is linear).
    Returns dict(status, obj, pobj, iters, x, z, y)."""
    ok, lb, ub, fmask = m.presolve(lbi, ubi)
    if not ok:
        return dict(status=2, obj=INF, pobj=np.nan, iters=0)
    mask = fmask[m.row_f]
    ce = check_every
    cost_int, const = m.cost_int, 0.0
    if m.dred:
        cost_int, const, m.lo[m.oD4], m.hi[m.oD4] = m.dred_terms(lb, ub)
    x = proj_simplex_rows(np.zeros((m.R, m.N)), mask)
    z = np.clip(np.zeros(m.n_int), lb, ub)
    y = np.zeros(m.n_dual)
    kz = m.K(x, z)
    xa, za, ya, kza = x.copy(), z.copy(), y.copy(), kz.copy()
    omega, eta = m.omega0, m.eta
    om_lo, om_hi = m.omega0 * 1e-5, m.omega0 * 1e5
    k = k_since = 0
    ks_base = -ce
    restart_pending = False
    last_fpr, prev_fpr = -1.0, INF
    best = -INF
    cost_x = m.row_wobj[:, None] * np.where(m.row_src[:, None] >= 0, m.D32[np.maximum(m.row_src, 0)], 0.0)
    block = 0
    while True:
        for it in range(ce):
            check, first = it == 0, it == 1
            plain = ce < 4 or it == 0 or it == ce - 1
            if first and restart_pending:
                xa, za, ya, kza = x.copy(), z.copy(), y.copy(), kz.copy()
            tau, sig = eta / omega, eta * omega
            gx, gz = m.KT(y)
            rcx = cost_x - gx
            rcz = cost_int - gz
            xn = proj_simplex_rows(x - tau * rcx, mask)
            zn = np.clip(z - tau * m.gam ** 2 * rcz, lb, ub)
            act = m.K(xn, zn)
            s = sig * m.rho ** 2
            V = y - s * (m.K(2 * xn - x, 2 * zn - z) if inline_reflect else 2 * act - kz)
            with np.errstate(invalid="ignore"):
                a = V + s * m.hi
                b = V + s * m.lo
            yn = np.where(a < 0, a, np.where(b > 0, b, 0.0))
            if check:
                lag = np.where(mask, rcx, INF).min(axis=1).sum()
                lag += np.where(rcz > 0, lb * rcz, ub * rcz).sum()
                with np.errstate(invalid="ignore"):
                    rl = np.where(y > 0, np.where(np.isfinite(m.lo), y * m.lo, -INF),
                                  np.where(y < 0, np.where(np.isfinite(m.hi), y * m.hi, -INF), 0.0))
                lag += rl.sum() + const
                pobj = (cost_x * xn).sum() + (cost_int * zn).sum() + const
                viol = np.maximum(np.maximum(m.lo - act, act - m.hi), 0.0) / m.rownorm
                res = viol.max()
                mvz = ((xn - x) ** 2).sum() + (((zn - z) / m.gam) ** 2).sum()
                mvy = (((yn - y) / m.rho) ** 2).sum()
                dsz = ((xn - xa) ** 2).sum() + (((zn - za) / m.gam) ** 2).sum()
                dsy = (((yn - ya) / m.rho) ** 2).sum()
            if plain:
                x, z, y, kz = xn, zn, yn, act
            else:
                ks = ks_base + it
                lam = (ks + 1.0) / (ks + 2.0)
                x = lam * (2 * xn - x) + (1 - lam) * xa
                z = lam * (2 * zn - z) + (1 - lam) * za
                y = lam * (2 * yn - y) + (1 - lam) * ya
                kz = lam * (2 * act - kz) + (1 - lam) * kza
            if check:
                k += 1 if block == 0 else ce
                k_since += 1 if block == 0 else ce
                restart_pending = False
                best = max(best, lag)
                gap = pobj - lag
                if verbose:
                    print(f"{k:7d} res={res:.2e} p={pobj:.10g} L={lag:.10g} gap={gap:.2e} w={omega:.3g}")
                if np.isfinite(lag) and res <= tol and gap <= tol * max(1.0, abs(lag)):
                    return dict(status=0, obj=lag, pobj=pobj, iters=k, x=x, z=z, y=y)
                if k >= max_iters:
                    return dict(status=1, obj=best, pobj=pobj, iters=k, x=x, z=z, y=y)
                fpr = np.sqrt(omega * mvz + mvy / omega)
                if last_fpr < 0:
                    last_fpr = fpr
                restart = (fpr <= 0.2 * last_fpr or (fpr <= 0.8 * last_fpr and fpr > prev_fpr)
                           or k_since >= 0.36 * k)
                prev_fpr = fpr
                if restart:
                    dz, dy = np.sqrt(dsz), np.sqrt(dsy)
                    if dz > 1e-10 and dy > 1e-10:
                        omega = float(np.clip(np.exp(0.5 * np.log(dy / dz) + 0.5 * np.log(omega)), om_lo, om_hi))
                    elif m.dred and dy > 1e-10:      # (reduced step 2: primal static -> weight x10, scalar_pass)
                        omega = float(min(omega * 10.0, om_hi))
                    restart_pending = True
                    k_since = 0
                    ks_base = -1
                    last_fpr = fpr
                    prev_fpr = INF
                else:
                    ks_base += ce
        block += 1
