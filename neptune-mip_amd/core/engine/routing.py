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
