"""ORACLE (test infrastructure only): the reference's MIP, restated as one CSR model.

Variable order (as the reference creates them):
  x[i,f,j]   `neptune/utils/variables.py:4-8`    index (f*N + i)*N + j   (f, then i, then j)
  c[f,j]     `variables.py:10-13`                 after x
  step 2:    moved_from, moved_to (`:19-27`), allocated, deallocated (`:29-33`)
  n[j]       `variables.py:15-17`                 last (step-1 MU/MDU; step-2 MU/MDU)
Row order follows the builder call order of the step classes:
  step 1  `neptune_step1.py:12-14,30-33,41-43` ; step 2 `neptune_step2.py:20-36,63-66,74-77,89-93`
Rows (`neptune/utils/constraints_step1.py`, `constraints_step2.py`):
  C1/C2 :5-15   C3 :18-23   C4 :27-34   C5 :57-65   C6/C7 :69-78   C8 :101-103
  D1 :5-9  D2 :12-16  D3 :19-33  D4 delete :36-44 / create :47-55
  D6 network delay :57-69   D5 node utilisation :71-73   D7 score :76-88
Objectives (`neptune/utils/objectives.py`): MinDelay :4-11, MinUtilization :24-27,
  MinDelayAndUtilization :30-52 (x terms only when total workload > 0), disruption :55-63.

The builders keep explicit zero coefficients (e.g. W == 0 terms); so does this CSR.
"""
import numpy as np
import scipy.sparse as sp

BIG_M = 10 ** 6          # constraints_step1.py:1
EPSILON = 10 ** -6       # constraints_step1.py:2
INF = np.inf

VARIANTS = ("MinDelay", "MinUtilization", "MinDelayAndUtilization")


class _Rows:
    def __init__(self):
        self.r, self.c, self.v, self.lo, self.hi = [], [], [], [], []
        self.n = 0

    def add_block(self, nrows, rows_local, cols, vals, lo, hi):
        self.r.append(np.asarray(rows_local, np.int64) + self.n)
        self.c.append(np.asarray(cols, np.int64))
        self.v.append(np.asarray(vals, np.float64))
        self.lo.append(np.broadcast_to(np.asarray(lo, np.float64), (nrows,)))
        self.hi.append(np.broadcast_to(np.asarray(hi, np.float64), (nrows,)))
        self.n += nrows

    def csr(self, nvars):
        r = np.concatenate(self.r) if self.r else np.zeros(0, np.int64)
        c = np.concatenate(self.c) if self.c else np.zeros(0, np.int64)
        v = np.concatenate(self.v) if self.v else np.zeros(0)
        A = sp.csr_matrix((v, (r, c)), shape=(self.n, nvars))
        A.sum_duplicates()
        return A, np.concatenate(self.lo), np.concatenate(self.hi)


def max_workload_delay(data):
    """objectives.py:36-43: sum_f sum_i W[f,i] * max{D[i,j'] : D[i,j'] <= maxdelay[f]} (loop order f, i)."""
    D, W, md = data.node_delay_matrix, data.workload_matrix, data.max_delay_matrix
    F, N = W.shape
    acc = 0
    for f in range(F):
        for i in range(N):
            acc += W[f, i] * max([d for d in D[i] if d <= md[f]])
    return acc


def score_max_delay(data):
    """constraints_step2.py:77-81: MD[i,f] = max(maxdelay[f], max_k D[k,i])."""
    D, md = data.node_delay_matrix, data.max_delay_matrix
    return np.maximum(md[None, :], D.max(axis=0)[:, None])


class Layout:
    def __init__(self, N, F, step, has_n):
        self.N, self.F, self.step, self.has_n = N, F, step, has_n
        self.nx = N * N * F
        self.nc = F * N
        self.c0 = self.nx
        if step == 1:
            self.n0 = self.nx + self.nc
            self.nvars = self.n0 + (N if has_n else 0)
        else:
            self.mf0 = self.nx + self.nc
            self.mt0 = self.mf0 + self.nc
            self.alloc = self.mt0 + self.nc
            self.dealloc = self.alloc + 1
            self.n0 = self.dealloc + 1
            self.nvars = self.n0 + (N if has_n else 0)

    def x(self, i, f, j):
        return (f * self.N + i) * self.N + j


def build_model(data, variant, step=1, mode="delete", alpha=0.5, soften_step1_sol=1.3, max_score=None,
                prev_x=None):
    """Return dict(A, lo, hi, c, lb, ub, integrality, layout) — the model the reference hands SCIP."""
    assert variant in VARIANTS
    D = data.node_delay_matrix
    W = data.workload_matrix
    F, N = W.shape
    has_n = variant in ("MinUtilization", "MinDelayAndUtilization")
    L = Layout(N, F, step, has_n)
    fi, ii, jj = np.meshgrid(np.arange(F), np.arange(N), np.arange(N), indexing="ij")  # [f,i,j]
    xidx = ((fi * N + ii) * N + jj)                                                    # == arange(nx)
    cidx = L.c0 + np.arange(F * N).reshape(F, N)
    rows = _Rows()

    # C1/C2 (constraints_step1.py:5-15), interleaved per (f, j)
    fj = np.arange(F * N)
    r1 = np.repeat(2 * fj, N + 1)
    cols1 = np.concatenate([xidx.transpose(0, 2, 1).reshape(F * N, N), cidx.reshape(-1, 1)], axis=1).ravel()
    v1 = np.tile(np.concatenate([np.ones(N), [-float(BIG_M)]]), F * N)
    v2 = np.tile(np.concatenate([np.ones(N), [-1.0]]), F * N)
    lo12 = np.empty(2 * F * N)
    hi12 = np.empty(2 * F * N)
    lo12[0::2], hi12[0::2] = -INF, 0.0
    lo12[1::2], hi12[1::2] = 0.0 - (0.0 + EPSILON), INF
    rows.add_block(2 * F * N, np.concatenate([r1, r1 + 1]), np.concatenate([cols1, cols1]),
                   np.concatenate([v1, v2]), lo12, hi12)

    # C3 memory (:18-23)
    mem_f = data.function_memory_matrix.astype(np.float64)
    rows.add_block(N, np.repeat(np.arange(N), F), cidx.T.ravel(), np.tile(mem_f, N),
                   -INF, data.node_memory_matrix.astype(np.float64))

    # C4 handle all requests (:27-34, ==1)
    rows.add_block(F * N, np.repeat(np.arange(F * N), N), xidx.reshape(-1), np.ones(F * N * N), 1.0, 1.0)

    # C5 CPU (:57-65): coef W[f,i] * cpr[f,j]
    cpr = data.core_per_req_matrix
    coef5 = (W.astype(np.float64)[:, :, None] * 1.0) * cpr[:, None, :]                  # [f,i,j]
    rows.add_block(N, jj.transpose(2, 0, 1).reshape(-1), xidx.transpose(2, 0, 1).reshape(-1),
                   coef5.transpose(2, 0, 1).reshape(-1), -INF, data.node_cores_matrix.astype(np.float64))

    def n_rows():
        # C6/C7 (:69-78) interleaved per node, then C8 budget (:101-103)
        nid = L.n0 + np.arange(N)
        r = np.repeat(2 * np.arange(N), F + 1)
        cols = np.concatenate([cidx.T, nid.reshape(-1, 1)], axis=1).ravel()
        va = np.tile(np.concatenate([np.ones(F), [-float(BIG_M)]]), N)
        vb = np.tile(np.concatenate([np.ones(F), [-1.0]]), N)
        lo = np.empty(2 * N)
        hi = np.empty(2 * N)
        lo[0::2], hi[0::2] = -INF, 0.0
        lo[1::2], hi[1::2] = 0.0 - (0.0 + EPSILON), INF
        rows.add_block(2 * N, np.concatenate([r, r + 1]), np.concatenate([cols, cols]),
                       np.concatenate([va, vb]), lo, hi)
        rows.add_block(N, np.arange(N), nid, data.node_costs.astype(np.float64), -INF, float(data.node_budget))

    obj = np.zeros(L.nvars)
    if step == 1:
        if has_n:
            n_rows()
        if variant == "MinDelay":
            obj[:L.nx] = (D[None, :, :] * W[:, :, None]).astype(np.float64).ravel()
        elif variant == "MinUtilization":
            obj[L.n0:L.n0 + N] = 1.0
        else:
            obj[L.n0:L.n0 + N] = float(alpha / N)
            if np.sum(W):
                mwd = max_workload_delay(data)
                obj[:L.nx] = (((1 - alpha) * W[:, :, None]) * D[None, :, :] / mwd).ravel()
    else:
        old = data.old_allocations_matrix
        sum_old = float(old.sum())
        mf = L.mf0 + np.arange(F * N)
        mt = L.mt0 + np.arange(F * N)
        cflat = cidx.ravel()
        oldf = old.ravel().astype(np.float64)
        k = np.arange(F * N)
        # D1 (:5-9): mf >= 0 ; mf - c >= -old   (interleaved per (f,j))
        rows.add_block(2 * F * N, np.concatenate([2 * k, 2 * k + 1, 2 * k + 1]),
                       np.concatenate([mf, mf, cflat]),
                       np.concatenate([np.ones(F * N), np.ones(F * N), -np.ones(F * N)]),
                       np.ravel(np.column_stack([np.zeros(F * N), -oldf])), INF)
        # D2 (:12-16): mt >= 0 ; mt + c >= old
        rows.add_block(2 * F * N, np.concatenate([2 * k, 2 * k + 1, 2 * k + 1]),
                       np.concatenate([mt, mt, cflat]), np.ones(3 * F * N),
                       np.ravel(np.column_stack([np.zeros(F * N), oldf])), INF)
        # D3 (:19-33)
        rows.add_block(1, [0], [L.alloc], [1.0], -INF, 0.0)
        rows.add_block(1, np.zeros(F * N + 1), np.concatenate([cflat, [L.alloc]]),
                       np.concatenate([-np.ones(F * N), [-1.0]]), -sum_old, INF)
        rows.add_block(1, [0], [L.dealloc], [1.0], -INF, 0.0)
        rows.add_block(1, np.zeros(F * N + 1), np.concatenate([cflat, [L.dealloc]]),
                       np.concatenate([np.ones(F * N), [-1.0]]), sum_old, INF)
        # D4 (:36-55)
        sgn = -1.0 if mode == "delete" else 1.0
        rows.add_block(1, np.zeros(F * N + 2), np.concatenate([[L.dealloc, L.alloc], cflat]),
                       np.concatenate([[1.0, 1.0], sgn * np.ones(F * N)]), sgn * sum_old, INF)
        if variant == "MinUtilization":
            n_rows()
            rows.add_block(1, np.zeros(N), L.n0 + np.arange(N), np.ones(N), -INF, max_score * soften_step1_sol)
        elif variant == "MinDelay":
            dw = (D[:, None, :] * W.T[:, :, None]).astype(np.float64)                    # [i,f,j]
            rhs = soften_step1_sol * np.sum((dw * prev_x).ravel())
            cols = xidx.transpose(1, 0, 2).ravel()                                          # (i,f,j) order
            rows.add_block(1, np.zeros(F * N * N), cols, dw.ravel(), -INF, rhs)
        else:
            n_rows()
            md = score_max_delay(data)                                                      # [i,f]
            coef = ((1 - alpha) * W.T[:, :, None]) * D[:, None, :] / md[:, :, None]        # [i,f,j]
            cols = np.concatenate([L.n0 + np.arange(N), xidx.transpose(1, 0, 2).ravel()])
            vals = np.concatenate([np.full(N, float(alpha / N)), coef.astype(np.float64).ravel()])
            rows.add_block(1, np.zeros(len(cols)), cols, vals, -INF, max_score * soften_step1_sol)
        w = float(old.size)
        obj[L.mf0:L.mf0 + F * N] = w
        obj[L.mt0:L.mt0 + F * N] = w
        obj[L.alloc] = w - 1
        obj[L.dealloc] = w + 1

    A, lo, hi = rows.csr(L.nvars)
    lb = np.zeros(L.nvars)
    ub = np.ones(L.nvars)
    integ = np.ones(L.nvars, np.int8)
    ub[:L.nx] = INF
    integ[:L.nx] = 0
    if step == 2:
        lb[L.alloc] = lb[L.dealloc] = -float(F * N)
        ub[L.alloc] = ub[L.dealloc] = 0.0
    return dict(A=A, lo=lo, hi=hi, c=obj, lb=lb, ub=ub, integrality=integ, layout=L, maximize=False, offset=0.0)


def facility_relaxation(m, data):
    """The B&B's strengthened relaxation (engine NEP_RELAX_FACILITY, include/neptune_lp.h) of a
    step-1 MinUtilization / MinDelayAndUtilization model `m` (build_model's dict): the big-M pairs C1/C2
    (constraints_step1.py:5-15) and C6/C7 (:69-78) are replaced by x[i,f,j] <= c[f,j] for every (i, f, j) and
    c[f,j] <= n[j] — valid for every integral placement (c = 0 forces the column's flow to 0 through C1; n = 0
    forces c = 0 through C6), and implying C1 and C6 for integral c, n; C2 / C7 (the eps floors) are relaxed;
    the capacity rows C3 / C5 take n[j] on their right-hand side (Mem_j n[j], cores_j n[j]: a closed node has
    neither memory nor CPU for anything).
    Test infrastructure: its HiGHS value is what the engine's facility LPs are checked against."""
    L = m["layout"]
    assert L.step == 1 and L.has_n, "step-1 MinUtilization / MinDelayAndUtilization only"
    N, F = L.N, L.F
    A = m["A"].tocsr()
    nrow = A.shape[0]
    keep = np.ones(nrow, bool)
    keep[:2 * F * N] = False                                    # C1/C2, interleaved per (f, j), built first
    coo = A.tocoo()
    big = (coo.col >= L.n0) & (coo.col < L.n0 + N) & ((coo.data == -float(BIG_M)) | (coo.data == -1.0))
    keep[np.unique(coo.row[big])] = False                       # C6/C7 (the rows with -M n / -n)
    # capacity rows scaled by n: C3 sum_f mem_f c[f,j] <= Mem_j n[j], C5 CPU_j <= cores_j n[j] (valid: an
    # integral n[j] = 0 closes every c[:, j] and x[:, :, j]); rows C3 / C5 are the first N rows after C1/C2 and
    # the N rows after C4 (build_model's order)
    r3 = 2 * F * N + np.arange(N)
    r5 = 2 * F * N + N + F * N + np.arange(N)
    cap = sp.csr_matrix((np.concatenate([-m["hi"][r3], -m["hi"][r5]]),
                         (np.concatenate([r3, r5]), np.concatenate([L.n0 + np.arange(N)] * 2))), shape=A.shape)
    A = (A + cap).tocsr()
    hi = m["hi"].copy()
    hi[r3] = 0.0
    hi[r5] = 0.0
    A, lo, hi = A[keep], m["lo"][keep], hi[keep]
    nv = A.shape[1]
    k = F * N * N
    r = np.arange(k)
    xc = sp.csr_matrix((np.concatenate([np.ones(k), -np.ones(k)]),
                        (np.concatenate([r, r]), np.concatenate([np.arange(k), L.c0 + (r // (N * N)) * N + r % N]))),
                       shape=(k, nv))
    q = np.arange(F * N)
    cn = sp.csr_matrix((np.concatenate([np.ones(F * N), -np.ones(F * N)]),
                        (np.concatenate([q, q]), np.concatenate([L.c0 + q, L.n0 + q % N]))), shape=(F * N, nv))
    A2 = sp.vstack([A, xc, cn]).tocsr()
    lo2 = np.concatenate([lo, np.full(k + F * N, -INF)])
    hi2 = np.concatenate([hi, np.zeros(k + F * N)])
    return dict(m, A=A2, lo=lo2, hi=hi2)
