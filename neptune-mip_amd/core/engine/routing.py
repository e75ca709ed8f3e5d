"""Sparse routing solution x[i][f][j] (reference `core/solvers/neptune/utils/output.py:5-21`
`output_x_and_c` reads it densely, N*F*N `solution_value()` calls).

The engine keeps the routing as aggregated rows (one per (function, loaded source) plus one pooled
row per function for all its zero-workload sources) and compacts a slot's nonzero
entries on the device (`nep_lp_routing_entries`): only (row, destination, value) triples cross
PCIe, never the dense N x F x N matrix (268 MB at 512x256, 2 GiB at 1024x512).  This object stands
in for the dense matrix where the reference keeps one (`Data.prev_x`, the step results):
  * `shape`, `size`, `np.asarray(r)` (dense on demand, for small instances and tests);
  * `entries()` — (i, f, j, value) of every nonzero in the dense matrix's C order (i, f, j), so the
    wire format built from it (`convert_x_matrix`) has the dense path's key order byte for byte;
  * `network_delay(D, W)` — sum D[i,j] W[f,i] x[i,f,j] (`constraints_step2.py:66-68`), from the
    loaded rows only (pooled rows carry W = 0).
"""
import numpy as np


class SparseRouting:
    def __init__(self, N, F, row_f, row_src, W, row, dst, val):
        self.N, self.F = int(N), int(F)
        self.row_f = np.asarray(row_f, np.int32)
        self.row_src = np.asarray(row_src, np.int32)
        self.zero_src = [np.flatnonzero(np.asarray(W, np.float64).reshape(F, N)[f] == 0) for f in range(F)]
        self.row = np.asarray(row, np.int32)
        self.dst = np.asarray(dst, np.int32)
        self.val = np.asarray(val, np.float64)

    @classmethod
    def empty(cls, N, F):
        z = np.zeros(0)
        return cls(N, F, z, z, np.ones((F, N)), z, z, z)

    @classmethod
    def from_dense(cls, x):
        """From a dense [i][f][j] matrix (one literal row per (f, i): no pooling)."""
        x = np.asarray(x, np.float64)
        N, F, _ = x.shape
        xr = x.transpose(1, 0, 2).reshape(F * N, N)
        row, dst = np.nonzero(xr)
        return cls(N, F, np.repeat(np.arange(F), N), np.tile(np.arange(N), F), np.ones((F, N)), row, dst,
                   xr[row, dst])

    shape = property(lambda self: (self.N, self.F, self.N))
    size = property(lambda self: self.N * self.F * self.N)
    ndim = 3

    def entries(self):
        """(i, f, j, value) of every stored nonzero, expanded over pooled rows, in (i, f, j) order."""
        f = self.row_f[self.row]
        src = self.row_src[self.row]
        loaded = src >= 0
        ii, ff, jj, vv = [src[loaded]], [f[loaded]], [self.dst[loaded]], [self.val[loaded]]
        for k in np.flatnonzero(~loaded):
            s = self.zero_src[f[k]]
            ii.append(s)
            ff.append(np.full(s.size, f[k], np.int32))
            jj.append(np.full(s.size, self.dst[k], np.int32))
            vv.append(np.full(s.size, self.val[k]))
        i, f, j, v = (np.concatenate(a) for a in (ii, ff, jj, vv))
        order = np.lexsort((j, f, i))
        return i[order], f[order], j[order], v[order]

    def __array__(self, dtype=None, copy=None):
        out = np.zeros(self.shape, np.float64 if dtype is None else dtype)
        i, f, j, v = self.entries()
        out[i, f, j] = v
        return out

    def network_delay(self, D, W):
        """sum D[i,j] W[f,i] x[i,f,j] over the loaded rows (pooled rows have W = 0)."""
        D = np.asarray(D, np.float64)
        W = np.asarray(W, np.float64).reshape(self.F, self.N)
        f = self.row_f[self.row]
        src = self.row_src[self.row]
        k = src >= 0
        return float(np.sum(D[src[k], self.dst[k]] * W[f[k], src[k]] * self.val[k]))

    def wire_entries(self, threshold=0.001):
        """Entries of the wire format (output.py:23-31): x > threshold, value np.round(x, 3)."""
        i, f, j, v = self.entries()
        keep = v > threshold
        return i[keep], f[keep], j[keep], np.round(v[keep], 3)

    def cpu_usage(self, W, cpr):
        """sum_{f,i} W[f,i] cpr[f,j] x[i,f,j] per destination j (constraints_step1.py:57-65), fp64."""
        W = np.asarray(W, np.float64).reshape(self.F, self.N)
        cpr = np.asarray(cpr, np.float64).reshape(self.F, self.N)
        f = self.row_f[self.row]
        src = self.row_src[self.row]
        k = src >= 0
        return np.bincount(self.dst[k], weights=self.val[k] * W[f[k], src[k]] * cpr[f[k], self.dst[k]],
                           minlength=self.N)


def repair_cpu(x, W, cpr, cores, c_open, coef=None, floor=1.0, max_moves=100000, score_room=None):
    """Make a leaf's routing meet the reference checker's CPU rows at an ABSOLUTE tolerance.

    The engine certifies C5 relative to the row norm; the reference's offline checker
    (`efttc/utils/constraints_step1.py:68-78`) accepts CPU_j <= cores_j + 1e-6 absolutely, so a
    certified routing can exceed a large node's cores by up to tol * rownorm (~1e-5).  The repair
    moves that excess flow of loaded rows (W > 0) from an overloaded destination j to another
    destination j' the placement opens for the same function (c[f, j'] = 1, so C1 holds) with CPU
    room, cheapest first by the change of `coef(f, i, j)` per unit of CPU relief; a source's row sum
    (C4) is unchanged, and j's column sum stays >= `floor` (C2 with c = 1) — every move is checked.
    Every overloaded node ends at CPU_j <= cores_j (not merely + 1e-6).

    x       SparseRouting of a leaf (every c fixed)
    c_open  [F, N] bool: the leaf's c
    coef    coef(f, i, j) -> the per-unit objective (or score-row) coefficient of x[i, f, j]
            (broadcasting arrays); None: every move costs 0
    score_room  step 2: how far the score / delay row (constraints_step2.py:57-88) may still rise,
            rhs + 1e-6 - activity (the reference checker's tolerance, efttc/utils/constraints_step2.py:
            55-95), with `coef` that row's x coefficients: a move is admissible only while the summed
            coefficient change of all moves stays within it (None: no such row)
    Returns (SparseRouting, sum of t * (coef(j') - coef(j)) over the moves, ok); ok = False when an
    overloaded node has no admissible move left (the routing is returned as far as repaired)."""
    F, N = x.F, x.N
    W = np.asarray(W, np.float64).reshape(F, N)
    cpr = np.asarray(cpr, np.float64).reshape(F, N)
    cores = np.asarray(cores, np.float64).reshape(N)
    c_open = np.asarray(c_open, bool).reshape(F, N)
    cpu = x.cpu_usage(W, cpr)
    lim = cores - 1e-12 * np.maximum(1.0, np.abs(cores))
    over = np.flatnonzero(cpu > cores)
    if over.size == 0:
        return x, 0.0, True
    row, dst, val = x.row.copy(), x.dst.copy(), x.val.copy()
    f_of, src_of = x.row_f, x.row_src
    weight = np.array([1.0 if s >= 0 else float(x.zero_src[f].size) for f, s in zip(f_of, src_of)])
    colsum = np.zeros(F * N)
    np.add.at(colsum, f_of[row] * N + dst, val * weight[row])
    where = {(int(r), int(d)): k for k, (r, d) in enumerate(zip(row, dst))}
    delta, ok, moves = 0.0, True, 0
    jj = np.arange(N)
    for j in over:
        while cpu[j] > lim[j] and moves < max_moves:
            ks = np.flatnonzero((dst == j) & (val > 0) & (src_of[row] >= 0))
            if ks.size == 0:
                ok = False
                break
            fk, ik = f_of[row[ks]], src_of[row[ks]]
            relief = W[fk, ik] * cpr[fk, j]
            cap_col = np.where(c_open[fk, j], colsum[fk * N + j] - floor, val[ks])
            cap = np.minimum(val[ks], cap_col)
            good = (relief > 0) & (cap > 0)
            if not good.any():
                ok = False
                break
            ks, fk, ik, relief, cap = ks[good], fk[good], ik[good], relief[good], cap[good]
            # destinations: open for f, not j, with CPU room
            load = W[fk, ik][:, None] * cpr[fk, :]                       # [K, N] CPU per unit at j'
            room = (lim - cpu)[None, :]
            cap_d = np.where(load > 0, np.where(room > 0, room / np.where(load > 0, load, 1.0), 0.0), np.inf)
            cap2 = np.minimum(cap[:, None], cap_d)
            adm = c_open[fk, :] & (jj[None, :] != j) & (cap2 > 1e-15)
            if not adm.any():
                ok = False
                break
            dc = np.zeros((ks.size, N)) if coef is None else \
                np.asarray(coef(fk[:, None], ik[:, None], jj[None, :]), np.float64) - \
                np.asarray(coef(fk, ik, np.full(ks.size, j)), np.float64)[:, None]
            tt = np.minimum(cap2, ((cpu[j] - lim[j]) / relief)[:, None])     # the move each candidate would make
            if score_room is not None:
                adm &= (dc <= 0.0) | (tt * dc <= max(0.0, score_room - delta))
                if not adm.any():
                    ok = False
                    break
            score = np.where(adm, dc / relief[:, None], np.inf)
            a, jd = np.unravel_index(int(np.argmin(score)), score.shape)
            t = float(tt[a, jd])
            k, f, i = int(ks[a]), int(fk[a]), int(ik[a])
            val[k] -= t
            key = (int(row[k]), int(jd))
            if key in where:
                val[where[key]] += t
            else:
                where[key] = len(val)
                row, dst, val = np.append(row, row[k]), np.append(dst, jd), np.append(val, t)
            cpu[j] -= t * relief[a]
            cpu[jd] += t * load[a, jd]
            colsum[f * N + j] -= t
            colsum[f * N + jd] += t
            delta += t * float(dc[a, jd])
            moves += 1
        if cpu[j] > lim[j]:
            ok = False
    keep = val > 0
    out = SparseRouting.__new__(SparseRouting)
    out.N, out.F, out.row_f, out.row_src, out.zero_src = N, F, x.row_f, x.row_src, x.zero_src
    out.row, out.dst, out.val = row[keep].astype(np.int32), dst[keep].astype(np.int32), val[keep]
    return out, delta, ok
