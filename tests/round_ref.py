"""Test reference (NOT product code): the branch-and-bound's rounding heuristic in the Python form
core/engine/bnb.py carried through round 4, kept so tests/test_round_native.py can hold the native
nep_round_leaf (csrc/nep_round.cpp) to the same leaves."""
import numpy as np


class RoundRef:
    def __init__(self, F, N, c0, c1, n_range, fn_mem, node_mem, flow_tol=1e-4):
        self.F, self.N, self.c0, self.c1, self.n_range = F, N, c0, c1, n_range
        self.fn_mem = np.asarray(fn_mem, np.float64).reshape(F)
        self.node_mem = np.asarray(node_mem, np.float64).reshape(N)
        self.flow_tol = flow_tol

    def _round(self, node, flow, zc=None, by_flow=True, min_flow=None):
        """Heuristic completion of a node (a leaf fixing every c and n), or None.

        Memory-aware greedy rounding of the node LP: the fixed c stay as fixed; the free c the LP
        holds at >= 1/2 (zc, the LP's c) are opened first, largest first, then the free (f, j) in
        decreasing order of the flow f sends to j, while node j's memory (C3,
        constraints_step1.py:18-23) has room and n[j] is not fixed to 0; a function left without an
        open destination gets the one with the largest LP c, then flow, that still has room;
        n[j] = any c[:, j] (a node fixed open gets its best-fitting function).  The leaf's LP then
        re-optimises x.  (Opening the LP's near-integral c first is what keeps step 2's placement
        next to the old allocation: its LP c sits at old wherever no flow forces a move.)
        by_flow=False skips the flow pass: the fewest openings the LP's c allows (a leaf whose x
        must then fit the CPU rows with those openings only).  min_flow: the flow pass opens only the
        (f, j) the LP already sends >= min_flow (an open (f, j) must receive >= 1 - eps, C2, so opening
        a trickle forces a unit of flow onto j's CPU; at 512x256 such leaves end CPU-infeasible)."""
        F, N, c0, c1 = self.F, self.N, self.c0, self.c1
        fixed = np.full(F * N, -1.0)
        sel = (node.idx >= c0) & (node.idx < c1)
        fixed[node.idx[sel] - c0] = node.val[sel]
        nfix = np.full(N, -1.0)
        if self.n_range is not None:
            n0, n1 = self.n_range
            seln = (node.idx >= n0) & (node.idx < n1)
            nfix[node.idx[seln] - n0] = node.val[seln]
        c = np.where(fixed > 0.5, 1.0, 0.0)
        cm = c.reshape(F, N)
        used = (self.fn_mem[:, None] * cm).sum(axis=0)
        room = self.node_mem + 1e-9
        if (used > room).any():
            return None
        fl = flow.ravel().astype(np.float64)
        closed = (fixed >= 0) | (np.repeat(nfix[None, :] == 0.0, F, axis=0).ravel())
        zc = np.zeros(F * N) if zc is None else np.asarray(zc, np.float64).ravel()
        usedl, rooml, fmem = used.tolist(), room.tolist(), self.fn_mem.tolist()

        def open_in_order(ks, key):
            """Greedy first-fit of the candidates ks (flat (f, j), ascending) into the node memories in
            decreasing `key` order (ties: lower index first).  A destination's decisions depend only on its
            own earlier ones: every destination whose candidates all fit takes them all (no sort); only the
            candidates of the few that fill up are sorted and walked."""
            if ks.size == 0:
                return
            fj, jj = np.divmod(ks, N)
            ms = self.fn_mem[fj]
            tot = np.bincount(jj, weights=ms, minlength=N)
            fit = tot <= np.asarray(rooml) - np.asarray(usedl)
            allin = fit[jj]
            opened = ks[allin].tolist()
            some = fit & (tot > 0)
            for j, u in zip(np.flatnonzero(some).tolist(), tot[some].tolist()):
                usedl[j] += u
            rest = ~allin
            if rest.any():
                kr, jr, mr, keyr = ks[rest], jj[rest], ms[rest], key[rest]
                o = np.lexsort((kr, -keyr, jr))          # by destination, then priority, then index
                for k, j, mq in zip(kr[o].tolist(), jr[o].tolist(), mr[o].tolist()):
                    if usedl[j] + mq <= rooml[j]:
                        opened.append(k)
                        usedl[j] += mq
            c[opened] = 1.0

        half = np.flatnonzero(~closed & (zc >= 0.5))
        open_in_order(half, zc[half])
        if by_flow:
            thr = self.flow_tol if min_flow is None else min_flow
            cand = np.flatnonzero(~closed & (c < 0.5) & (fl > thr))
            open_in_order(cand, fl[cand])
        need = np.flatnonzero(cm.sum(axis=1) < 1)
        if need.size:
            # each function left without a destination: the open-able destination with the largest LP c,
            # then flow (lowest index on ties), or the next one in that order that still has room
            ZC, FL, CL = zc.reshape(F, N)[need], fl.reshape(F, N)[need], closed.reshape(F, N)[need]
            zcm = np.where(CL, -np.inf, ZC)
            top = zcm.max(axis=1)
            first = np.where(CL | (zcm < top[:, None]), -np.inf, FL).argmax(axis=1).tolist()
            opened = []
            for r, f in enumerate(need.tolist()):
                if top[r] == -np.inf:
                    return None
                j = first[r]
                if usedl[j] + fmem[f] > rooml[j]:
                    order = np.lexsort((-FL[r], -ZC[r]))
                    j = next((jj for jj in order[~CL[r][order]].tolist() if usedl[jj] + fmem[f] <= rooml[jj]), None)
                    if j is None:
                        return None
                opened.append(f * N + j)
                usedl[j] += fmem[f]
            c[opened] = 1.0
        used = np.asarray(usedl)
        idx = [np.arange(c0, c1)]
        val = [c]
        if self.n_range is not None:
            nv = (cm.sum(axis=0) >= 1).astype(np.float64)
            for j in np.flatnonzero((nfix == 1.0) & (nv == 0.0)):
                fs = [f for f in np.argsort(self.fn_mem, kind="stable")
                      if fixed[f * N + j] < 0 and used[j] + self.fn_mem[f] <= room[j]]
                if not fs:
                    return None
                c[fs[0] * N + j] = 1.0
                used[j] += self.fn_mem[fs[0]]
                nv[j] = 1.0
            if ((nfix == 0.0) & (nv == 1.0)).any():
                return None
            idx.append(np.arange(n0, n1))
            val.append(nv)
        return np.concatenate(idx), np.concatenate(val)
