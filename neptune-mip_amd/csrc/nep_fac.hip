// nep_fac.hip — gfx950 PDHG passes of the facility relaxation (NEP_RELAX_FACILITY, include/neptune_lp.h).
//
// The step-1 model with x[r, j] <= c[f, j] on every routing row and c[f, j] <= n[j] in place of the big-M
// pairs C1/C2 and C6/C7: a strengthened relaxation — valid for every integral placement, no 1e6 / 1e-6
// coefficients — that the branch-and-bound bounds its nodes with.  Same iteration as
// nep_kernels.hip (reflected restarted Halpern PDHG, diagonal preconditioning, routing rows kept on their
// simplexes), same certificate protocol (scalar_pass), different rows:
//   fac_x_pass     one workgroup per (function f, slot): first c[f, :] — its T step needs only the previous
//                  iteration's duals (memory y3, the c <= n duals mu, and per (f, j) the sum over the rows of
//                  f of the x <= c duals lambda, kept from the previous pass) — then every routing row of f:
//                  the gradient with lambda[r, :], the simplex projection, lambda's dual step with the
//                  reflected x and c, the Halpern combination of both, the CPU shares;
//   fac_node_pass  per node: n, the memory (C3) and CPU (C5) rows (capacities Mem_j n, cores_j n), then the
//                  c <= n duals of every f.
// Certificate point: x̂ with the least c every row allows (c = max_r x̂[r, j]) and the least n (max_f c).
// Reference rows: constraints_step1.py:18-23 (C3), :27-34 (C4), :57-65 (C5), :101-103 (C8); the cuts hold for
// the binaries of :5-15 and :69-78.  Objective objectives.py:24-53.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <algorithm>
#include <cmath>

#include "nep_internal.h"
#include "nep_device.h"

namespace nep {

template <int CPL, bool CHECK, bool INIT, bool FIRST, int TW>
__global__ __launch_bounds__(kWave * TW) __attribute__((amdgpu_waves_per_eu(CHECK ? 2 : (CPL >= 8 ? 2 : (CPL >= 4 ? 3 : 4)), 8)))
void fac_x_pass(DeviceView v, const int32_t *__restrict__ slots, int plain, int it, int nslots, int nt_i) {
  const bool nt = nt_i != 0;
  constexpr int E = 4 * CPL;
  constexpr int SW = CHECK ? 2 : 1;   // words per CPU-sum accumulator (fp64 on certificate launches)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ double lds_s[TW][NTS + NBS];
  __shared__ double lds0[TW][4];      // the c step's partials per wave (certificate launches)
  // XCD-aware order, as x_pass: the slots of one function back to back on one XCD (its delay rows stay in L2)
  const int total = v.F * nslots, Q = (total + 7) / 8;
  const int p = (int)(blockIdx.x % 8) * Q + (int)(blockIdx.x / 8);
  if (p >= total) return;
  const int f = p / nslots;
  const int slot = slots[p - f * nslots];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int NP = v.NP, F = v.F, N = v.N;
  const double taud = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const float tau = (float)taud;
  const bool restart = INIT || (FIRST && ctrl->restart_pending);
  const bool halp = !INIT && !plain;
  const double lamd = halpern_lambda(ctrl, halp, it);
  const float lam = (float)lamd;
  const bool need_anchor = (halp || CHECK) && !restart;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r0 = v.frow[f], nrows = v.frow[f + 1] - r0;
  float *__restrict__ x = v.x + slot * v.sx;
  float *__restrict__ xa = v.xa + slot * v.sx;
  float *__restrict__ lm = v.lam + slot * v.sx;      // x <= c duals, [R][NP] like x
  float *__restrict__ lma = v.lama + slot * v.sx;    // their anchor
  int32_t *__restrict__ acnt = v.acnt + (int64_t)slot * v.R;
  AnchorEnt *__restrict__ aent = v.aent + ((int64_t)slot * v.R) * kAnchorK;
  float *__restrict__ th_row = v.theta + (int64_t)slot * v.R;
  const uint8_t *__restrict__ mask = v.mask + slot * v.smask + (int64_t)f * NP;
  const float *__restrict__ kty = v.kty + slot * v.skty;
  float *__restrict__ lsum = v.lsum + slot * v.slsum + (int64_t)f * NP;
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  const double *y = v.y + slot * v.sdual;

  // LDS: per-wave CPU sums lW [SW][TW][NP], per-wave sums of the new lambda lL [TW][NP] (f32), per-wave column
  // max of x̂ lX [TW][NP] (f32, certificate launches); per j: lC = cpr y5, lR = 2ĉ - c, lS = sigma rho_L^2 (f32);
  // lCh = ĉ, lRd = 2ĉ - c, lCd = cpr y5 (f64; lCd on certificate launches)
  float *lW = lds;
  double *lWd = reinterpret_cast<double *>(lW);
  float *lL = lW + SW * TW * NP;
  float *lX = lL + TW * NP;
  float *lC = lX + (CHECK ? TW * NP : 0);
  float *lR = lC + NP, *lS = lR + NP;
  double *lCh = reinterpret_cast<double *>(lS + NP);
  double *lRd = lCh + NP, *lCd = lRd + NP;

  // stage 0: c[f, :].  Reduced cost cost - K^T y with C3 (mem_f y3), the x <= c rows of f (-sum_r lambda) and
  // the c <= n row (mu); every dual is the previous iteration's, so ĉ is known before the rows (PDHG's order)
  SmallAcc a0;
  for (int j = threadIdx.x; j < NP; j += kWave * TW) {
    if (j < N) {
      const int idx = f * N + j, k = il.oc + idx;
      const double rc = v.cost_int[k] - (v.mem_f[f] * y[dl.o3 + j] - (double)lsum[j] + y[dl.oQ + idx]);
      const double c_old = zi[k];
      const double ch = primal_step<CHECK>(v, zi, zia, lb, ub, k, rc, taud, restart, halp, lamd, a0);
      lCh[j] = ch;
      lRd[j] = 2.0 * ch - c_old;
      lR[j] = (float)(2.0 * ch - c_old);
      const double rl = v.rho_l[(int64_t)f * NP + j];
      lS[j] = (float)(sigma * rl * rl);
      lC[j] = v.cpr[(int64_t)f * NP + j] * kty[(int64_t)F * NP + j];
      if (CHECK) lCd[j] = (double)v.cpr[(int64_t)f * NP + j] * y[dl.o5 + j];
    } else {
      lCh[j] = lRd[j] = 0.0;
      lR[j] = lS[j] = lC[j] = 0.f;
      if (CHECK) lCd[j] = 0.0;
    }
  }
  if (CHECK) {
    const double t0 = wave_sum_d(a0.lagr), t1 = wave_sum_d(a0.lagr0), t2 = wave_sum_d(a0.mvz), t3 = wave_sum_d(a0.dsz);
    if (lane == 0) {
      lds0[wave][0] = t0;
      lds0[wave][1] = t1;
      lds0[wave][2] = t2;
      lds0[wave][3] = t3;
    }
  }
  uint32_t mbits = 0;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j0 = 4 * (lane + kWave * q);
    if (j0 < NP) {
      const uchar4 mk = *reinterpret_cast<const uchar4 *>(mask + j0);
      mbits |= (uint32_t)(mk.x != 0) << (4 * q) | (uint32_t)(mk.y != 0) << (4 * q + 1) |
               (uint32_t)(mk.z != 0) << (4 * q + 2) | (uint32_t)(mk.w != 0) << (4 * q + 3);
      if (CHECK) {
        double2 *pe = reinterpret_cast<double2 *>(lWd + wave * NP + j0);
        pe[0] = pe[1] = make_double2(0.0, 0.0);
        *reinterpret_cast<float4 *>(lX + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        *reinterpret_cast<float4 *>(lW + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      *reinterpret_cast<float4 *>(lL + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  int cnt_f = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) cnt_f += __popcll(__ballot((mbits >> e) & 1u));

  double s_pobj = 0.0, s_lagr = 0.0, s_lagr0 = 0.0, s_move = 0.0, s_dist = 0.0, s_mvy = 0.0, s_dsy = 0.0;
  const double s_empty = (cnt_f == 0 && threadIdx.x == 0) ? (double)nrows : 0.0;

  for (int rr = wave; rr < nrows; rr += TW) {
    const int r = r0 + rr;
    const RowInfo ri = v.rows[r];
    const bool nd = ri.src >= 0 && ri.wobj != 0.f;
    float xc[E], dc[E], ac[E];
    int acn = 0;
    if (need_anchor) acn = NEP_SPARSE_ANCHOR ? __builtin_amdgcn_readfirstlane(acnt[r]) : kAnchorDense;
    load_row<CPL>(x + (int64_t)r * NP, v.D + (int64_t)(ri.src < 0 ? 0 : ri.src) * NP, xa + (int64_t)r * NP, nd,
                  need_anchor && acn > kAnchorK, nt, lane, NP, xc, dc, ac);
    if (need_anchor && acn <= kAnchorK) {
      AnchorEnt ae{0, 0.f};
      if (lane < acn) ae = aent[(int64_t)r * kAnchorK + lane];
      for (int k = 0; k < acn; ++k) {
        const int jk = __builtin_amdgcn_readlane(ae.j, k);
        const float vk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ae.v), k));
        const int ek = ((jk >> 8) << 2) | (jk & 3);
        const bool mine = lane == ((jk >> 2) & (kWave - 1));
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (e == ek) ac[e] = mine ? vk : ac[e];
      }
    }
    // the row's x <= c duals and (Halpern / restart distance) their anchor
    float lv[E], la[E];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      f32x4 t = {0.f, 0.f, 0.f, 0.f}, u = t;
      if (j0 < NP) {
        t = ld_x4(lm + (int64_t)r * NP + j0, nt);
        if (need_anchor) u = ld_x4(lma + (int64_t)r * NP + j0, nt);
      }
      lv[4 * q] = t.x; lv[4 * q + 1] = t.y; lv[4 * q + 2] = t.z; lv[4 * q + 3] = t.w;
      la[4 * q] = u.x; la[4 * q + 1] = u.y; la[4 * q + 2] = u.z; la[4 * q + 3] = u.w;
    }
    const float w = ri.w, wobj = ri.wobj;
    float vv[E];
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = 4 * (lane + kWave * (e / 4)) + (e & 3);
      const float cy5 = j < NP ? lC[j] : 0.f;
      const float g = wobj * dc[e] - (w * cy5 + lv[e]);
      vv[e] = xc[e] - tau * g;
      if ((mbits >> e) & 1u) s += vv[e];
    }
    if (CHECK) {
      // the row's Lagrangian term: min over its simplex of the reduced cost (fp64; at the objective off: L0)
      double gmin = INFINITY, gmin0 = INFINITY;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((mbits >> e) & 1u) {
          const int j = 4 * (lane + kWave * (e / 4)) + (e & 3);
          const double gx = -((double)w * lCd[j] + (double)lv[e]);
          gmin = fmin(gmin, (double)wobj * dc[e] + gx);
          gmin0 = fmin(gmin0, gx);
        }
      }
      gmin = wave_min_d(gmin);
      gmin0 = wave_min_d(gmin0);
      if (lane == 0) { s_lagr += gmin; s_lagr0 += gmin0; }
    }
    // projection onto the row's simplex (x_pass's safeguarded Michelot iteration, from the row's last threshold)
    float theta = INFINITY;
    if (cnt_f > 0) {
      float vm = -INFINITY;
#pragma unroll
      for (int e = 0; e < E; ++e)
        if ((mbits >> e) & 1u) vm = fmaxf(vm, vv[e]);
      const float th0 = th_row[r];
      float lo_s = 0.f;
      int lo_c = 0;
      if (!INIT && th0 > -INFINITY && th0 < INFINITY) {
        float s0 = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool in = ((mbits >> e) & 1u) && vv[e] > th0;
          if (in) s0 += vv[e];
          lo_c += __popcll(__ballot(in));
        }
        lo_s = wave_sum_u(s0);
      }
      if (lo_c == 0) {
        lo_s = wave_sum_u(s);
        lo_c = cnt_f;
      }
      float hi = INFINITY;
      float lo = -INFINITY;
      for (int k = 0; k < 96; ++k) {
        const bool bisect = k >= 4 && (k & 1) && lo > -INFINITY;
        if (bisect && hi == INFINITY) hi = wave_max_u(vm);
        const float t = bisect ? 0.5f * (lo + hi) : (lo_s - 1.f) / (float)lo_c;
        float s2 = 0.f;
        int c2 = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool in = ((mbits >> e) & 1u) && vv[e] > t;
          if (in) s2 += vv[e];
          c2 += __popcll(__ballot(in));
        }
        s2 = wave_sum_u(s2);
        if (!bisect) {
          theta = t;
          if (c2 == lo_c || c2 == 0) break;
          lo = t; lo_s = s2; lo_c = c2;
        } else if (s2 - t * (float)c2 - 1.f >= 0.f && c2 > 0) {
          lo = t; lo_s = s2; lo_c = c2;
        } else {
          hi = t;
        }
      }
    }
    if (lane == 0) th_row[r] = theta;
    float xn[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xn[e] = ((mbits >> e) & 1u) ? fmaxf(vv[e] - theta, 0.f) : 0.f;
    float xav[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xav[e] = need_anchor ? ac[e] : (INIT ? xn[e] : xc[e]);
    if (CHECK && !restart) {
      double dd = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) { const double t = (double)xn[e] - xav[e]; dd += t * t; }
      s_dist += dd;
    }
    // store x, and lambda's dual step: y' = prox(y - sigma rho^2 K(2ŵ - w)) on its row x - c <= 0, with the
    // reflected activity (2x̂ - x)[r, j] - (2ĉ - c)[f, j]; the Halpern combination as for x
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      if (j0 < NP) {
        float o[4], ln[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int e = 4 * q + t, j = j0 + t;
          o[t] = halp ? lam * (2.f * xn[e] - xc[e]) + (1.f - lam) * xav[e] : xn[e];
          const float lanc = need_anchor ? la[e] : lv[e];   // (at a restart the anchor is the current iterate)
          float lnew = lv[e];
          if (!INIT) {
            const float d = (2.f * xn[e] - xc[e]) - lR[j];
            const float lh = fminf(0.f, lv[e] - lS[j] * d);
            lnew = halp ? lam * (2.f * lh - lv[e]) + (1.f - lam) * lanc : lh;
            if (CHECK && lS[j] > 0.f) {
              const double inv = sigma / (double)lS[j];   // 1 / rho^2
              const double dm = (double)lh - lv[e], du = (double)lh - lanc;
              s_mvy += dm * dm * inv;
              s_dsy += du * du * inv;
            }
          }
          ln[t] = lnew;
        }
        st_x4(x + (int64_t)r * NP + j0, f32x4{o[0], o[1], o[2], o[3]}, nt);
        if (!INIT) st_x4(lm + (int64_t)r * NP + j0, f32x4{ln[0], ln[1], ln[2], ln[3]}, nt);
        if (restart)
          st_x4(lma + (int64_t)r * NP + j0, f32x4{lv[4 * q], lv[4 * q + 1], lv[4 * q + 2], lv[4 * q + 3]}, nt);
        float4 *pl = reinterpret_cast<float4 *>(lL + wave * NP + j0);
        float4 cl = *pl;
        cl.x += ln[0]; cl.y += ln[1]; cl.z += ln[2]; cl.w += ln[3];
        *pl = cl;
      }
    }
    if (restart) {
      // x's new anchor: (j, value) pairs when it has <= kAnchorK nonzeros, else dense (as x_pass)
      int tot = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) tot += __popcll(__ballot(4 * (lane + kWave * (e / 4)) < NP && xav[e] != 0.f));
      if (NEP_SPARSE_ANCHOR && tot <= kAnchorK) {
        int base = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool nz = 4 * (lane + kWave * (e / 4)) < NP && xav[e] != 0.f;
          const uint64_t b = __ballot(nz);
          if (nz) {
            const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            aent[(int64_t)r * kAnchorK + pos] = AnchorEnt{4 * (lane + kWave * (e / 4)) + (e & 3), xav[e]};
          }
          base += __popcll(b);
        }
      } else {
        tot = kAnchorDense;
        float *arow = xa + (int64_t)r * NP;
#pragma unroll
        for (int q = 0; q < CPL; ++q) {
          const int j0 = 4 * (lane + kWave * q);
          if (j0 < NP) st_x4(arow + j0, f32x4{xav[4 * q], xav[4 * q + 1], xav[4 * q + 2], xav[4 * q + 3]}, nt);
        }
      }
      if (lane == 0) acnt[r] = tot;
    }
    // CPU shares (C5) and, on certificate launches, the column max of x̂ (the least c the row allows)
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      if (j0 < NP) {
        const float *xq = xn + 4 * q;
        if (CHECK) {
          double2 *pe = reinterpret_cast<double2 *>(lWd + wave * NP + j0);
          double2 b0 = pe[0], b1 = pe[1];
          const double wd = w;
          b0.x += wd * xq[0]; b0.y += wd * xq[1]; b1.x += wd * xq[2]; b1.y += wd * xq[3];
          pe[0] = b0; pe[1] = b1;
          float4 *px = reinterpret_cast<float4 *>(lX + wave * NP + j0);
          float4 mx = *px;
          mx.x = fmaxf(mx.x, xq[0]); mx.y = fmaxf(mx.y, xq[1]); mx.z = fmaxf(mx.z, xq[2]); mx.w = fmaxf(mx.w, xq[3]);
          *px = mx;
        } else {
          float4 *pw = reinterpret_cast<float4 *>(lW + wave * NP + j0);
          float4 b = *pw;
          b.x += w * xq[0]; b.y += w * xq[1]; b.z += w * xq[2]; b.w += w * xq[3];
          *pw = b;
        }
      }
    }
    if (CHECK) {
      double po = 0.0, mv = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        po += (double)dc[e] * xn[e];
        const double t = (double)xn[e] - xc[e];
        mv += t * t;
      }
      s_pobj += (double)wobj * po;
      s_move += mv;
    }
  }
  __syncthreads();

  // per (f, j): the wave reductions (fixed order), f's shares of the node rows and the certificate's c
  double *np_ = v.npart + slot * v.snpart + (int64_t)f * 3 * NP;
  SmallAcc a;
  for (int j = threadIdx.x; j < N; j += kWave * TW) {
    float Lf = 0.f, Uf = 0.f, Xm = 0.f;
    double Ud = 0.0;
#pragma unroll
    for (int wv = 0; wv < TW; ++wv) {
      Lf += lL[wv * NP + j];
      if (CHECK) {
        Ud += lWd[wv * NP + j];
        Xm = fmaxf(Xm, lX[wv * NP + j]);
      } else {
        Uf += lW[wv * NP + j];
      }
    }
    lsum[j] = Lf;   // sum over the rows of f of the new lambda: c's reduced cost at the next iteration
    const double cp = v.cpr[(int64_t)f * NP + j];
    np_[j] = lCh[j];                                // node_pass forms the memory share mem_f * ĉ
    np_[NP + j] = CHECK ? Ud * cp : (double)(Uf * (float)cp);
    np_[2 * NP + j] = lRd[j];                       // reflected c for the c <= n duals
    if (CHECK) {
      // repaired c: the least value every routing row of f allows (c >= x̂[r, j]) within the node box
      const int k = il.oc + f * N + j;
      const double cr = fmax(lb[k], (double)Xm);
      a.res = fmax(a.res, cr - ub[k]);            // absolute: flow where the box closes c
      a.pobj += v.cost_int[k] * cr;
      v.zr[slot * v.sint + k] = cr;
      double *rp = v.rpart + slot * v.srpart + (int64_t)f * 2 * NP;
      rp[j] = v.mem_f[f] * cr;
      rp[NP + j] = cr;
    }
  }
  if (!(INIT || CHECK)) return;
  double vals[NTS + NBS];
#pragma unroll
  for (int k = 0; k < NTS + NBS; ++k) vals[k] = 0.0;
  vals[TS_POBJ] = s_pobj;
  vals[TS_LAGR] = s_lagr;
  vals[TS_MOVE] = s_move;
  vals[TS_DIST] = s_dist;
  vals[TS_EMPTY] = s_empty;
  vals[TS_LAGR0] = s_lagr0;
  vals[NTS + BS_POBJ] = a.pobj;
  vals[NTS + BS_RES] = a.res;
  vals[NTS + BS_MOVE_Y] = s_mvy;
  vals[NTS + BS_DIST_Y] = s_dsy;
  constexpr int NW = NTS + NBS;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const double t = (k == NTS + BS_RES) ? wave_max_d(vals[k]) : wave_sum_d(vals[k]);
    if (lane == 0) lds_s[wave][k] = t;
  }
  __syncthreads();
  const int k = threadIdx.x;
  if (k < NW) {
    double t = 0.0;
#pragma unroll
    for (int wv = 0; wv < TW; ++wv) t = (k == NTS + BS_RES) ? fmax(t, lds_s[wv][k]) : t + lds_s[wv][k];
    if (CHECK) {   // the c step's terms (stage 0)
#pragma unroll
      for (int wv = 0; wv < TW; ++wv) {
        if (k == NTS + BS_LAGR) t += lds0[wv][0];
        if (k == NTS + BS_LAGR0) t += lds0[wv][1];
        if (k == NTS + BS_MOVE_Z) t += lds0[wv][2];
        if (k == NTS + BS_DIST_Z) t += lds0[wv][3];
      }
    }
    if (k < NTS) v.tpart[slot * v.stpart + (int64_t)f * NTS + k] = t;
    else v.bpart[slot * v.sbpart + (int64_t)f * NBS + (k - NTS)] = t;
  }
}

// One workgroup per (slot, block of kNodeJ nodes): the function shares of the node rows (fixed order), then
// wave 0 updates n, C3 and C5, then every thread the c <= n duals of its functions at its node.
template <bool CHECK, bool INIT>
__global__ __launch_bounds__(kNodeThreads) void fac_node_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                              int plain, int it) {
  constexpr int NG = kNodeThreads / kNodeJ;
  __shared__ double red[5][NG][kNodeJ];
  __shared__ double nref[kNodeJ];
  const int jb = blockIdx.x;
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  const int NP = v.NP, F = v.F, N = v.N;
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  const bool copy_anchor = INIT || (first && ctrl->restart_pending);
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  const double tau = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool halp = !INIT && !plain;
  const double lam = halpern_lambda(ctrl, halp, it);
  const double *npart = v.npart + slot * v.snpart;
  const int j = jb * kNodeJ + lane;
  const bool valid = wave == 0 && lane < kNodeJ && j < N;
  DPre p3{}, p5{};
  ZPre pn{};
  double nrm3 = 1.0, nrm5 = 1.0;
  if (valid) {
    p3 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o3 + j, copy_anchor);
    p5 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o5 + j, copy_anchor);
    pn = primal_pre(v, zi, zia, lb, ub, il.on + j, copy_anchor);
    if (CHECK) {
      nrm3 = v.rownorm[dl.o3 + j];
      nrm5 = v.rownorm[dl.o5 + j];
    }
  }
  const int jj = threadIdx.x % kNodeJ, g = threadIdx.x / kNodeJ;
  const int jl = jb * kNodeJ + jj;
  const int per = (F + NG - 1) / NG;
  const int f0 = g * per, f1 = min(F, f0 + per);
  {
    double memc = 0.0, U = 0.0, musum = 0.0, memr = 0.0, cmax = 0.0;
    if (jl < N) {
      for (int f = f0; f < f1; ++f) {
        const double *pf = npart + (int64_t)f * 3 * NP;
        memc += __dmul_rn(v.mem_f[f], pf[jl]);
        U += pf[NP + jl];
        musum += y[dl.oQ + f * N + jl];
      }
      if (CHECK) {
        const double *rp = v.rpart + slot * v.srpart;
        for (int f = f0; f < f1; ++f) {
          memr += rp[(int64_t)f * 2 * NP + jl];
          cmax = fmax(cmax, rp[(int64_t)f * 2 * NP + NP + jl]);
        }
      }
    }
    red[0][g][jj] = memc;
    red[1][g][jj] = U;
    red[2][g][jj] = musum;
    red[3][g][jj] = memr;
    red[4][g][jj] = cmax;
  }
  __syncthreads();
  SmallAcc a;
  if (valid) {
    double memc = 0.0, U = 0.0, musum = 0.0, memr = 0.0, cmax = 0.0;
#pragma unroll 8
    for (int q = 0; q < NG; ++q) {
      memc += red[0][q][lane];
      U += red[1][q][lane];
      musum += red[2][q][lane];
      if (CHECK) {
        memr += red[3][q][lane];
        cmax = fmax(cmax, red[4][q][lane]);
      }
    }
    // n[j] first (its T step prices the rows at the old duals): the c <= n rows give it the coefficient -1
    // each, C3 -Mem_j and C5 -cores_j, so its reduced cost is cost_n + sum_f mu[f, j] + Mem_j y3 + cores_j y5
    const double capM = v.capn[j], capC = v.capn[N + j];
    const double n_old = pn.z;
    const double nn = primal_step_p<CHECK>(zi, zia, il.on + j, pn.cost + musum + capM * p3.y + capC * p5.y, pn, tau,
                                           copy_anchor, halp, lam, a);
    nref[lane] = 2.0 * nn - n_old;
    if (CHECK) {   // repaired n: the least value the repaired c (n >= c, Mem_j n >= its memory) and x̂ (cores_j
                   // n >= its CPU) allow, within the node box; C3 / C5 at that point
      double nr = fmax(pn.lb, cmax);
      if (capM > 0.0) nr = fmax(nr, memr / capM);
      if (capC > 0.0) nr = fmax(nr, U / capC);
      a.res = fmax(a.res, nr - pn.ub);
      nr = fmin(nr, pn.ub);
      a.res = fmax(a.res, row_viol(memr - capM * nr, p3.lo, p3.hi) / nrm3);
      a.res = fmax(a.res, row_viol(U - capC * nr, p5.lo, p5.hi) / nrm5);
      a.pobj += pn.cost * nr;
      v.zr[slot * v.sint + il.on + j] = nr;
    }
    // C3 / C5 at (ĉ, x̂, n̂)
    dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o3 + j, memc - capM * nn, p3, sigma, copy_anchor, halp, lam, a);
    const double y5n =
        dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o5 + j, U - capC * nn, p5, sigma, copy_anchor, halp, lam, a);
    v.kty[slot * v.skty + (int64_t)F * NP + j] = (float)y5n;
  }
  __syncthreads();
  // the c <= n duals mu[f, j] of this node block: reflected activity (2ĉ - c) - (2n̂ - n); their Lagrangian
  // row terms are 0 (right-hand side 0, mu <= 0)
  double mvy = 0.0, dsy = 0.0;
  if (jl < N) {
    for (int f = f0; f < f1; ++f) {
      const int row = dl.oQ + f * N + jl;
      const double mu = y[row];
      const double mua = copy_anchor ? mu : ya[row];
      if (copy_anchor) ya[row] = mu;
      if (!INIT) {
        const double rr = v.rho[row];
        const double d = npart[(int64_t)f * 3 * NP + 2 * NP + jl] - nref[jj];
        const double mh = dual_prox(mu, sigma * rr * rr, d, v.lo[row], v.hi[row]);
        const double t = (mh - mu) / rr;
        mvy += t * t;
        if (CHECK) { const double u = (mh - mua) / rr; dsy += u * u; }
        y[row] = halp ? lam * (2.0 * mh - mu) + (1.0 - lam) * mua : mh;
      }
    }
  }
  red[0][g][jj] = mvy;
  red[1][g][jj] = dsy;
  __syncthreads();
  if (wave != 0) return;
  if (lane < kNodeJ) {
#pragma unroll 8
    for (int q = 0; q < NG; ++q) {
      a.mvy += red[0][q][lane];
      a.dsy += red[1][q][lane];
    }
  }
  if (CHECK || INIT) {
    double vals[NBS];
#pragma unroll
    for (int k = 0; k < NBS; ++k) vals[k] = 0.0;
    vals[BS_LAGR] = a.lagr;
    vals[BS_POBJ] = a.pobj;
    vals[BS_RES] = a.res;
    vals[BS_MOVE_Z] = a.mvz;
    vals[BS_MOVE_Y] = a.mvy;
    vals[BS_DIST_Z] = a.dsz;
    vals[BS_DIST_Y] = a.dsy;
    vals[BS_LAGR0] = a.lagr0;
    double *bp = v.bpart + slot * v.sbpart + ((int64_t)F + jb) * NBS;
#pragma unroll
    for (int k = 0; k < NBS; ++k) {
      const double t = (k == BS_RES) ? wave_max_d(vals[k]) : wave_sum_d(vals[k]);
      if (lane == 0) bp[k] = t;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
static size_t fac_lds_bytes(int tw, int NP, bool check) {
  const int sw = check ? 2 : 1;
  return (size_t)(sw * tw + tw + (check ? tw : 0) + 3) * NP * sizeof(float) + 3 * (size_t)NP * sizeof(double);
}

template <int CPL, int TW>
static hipError_t launch_fac_tw(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                                bool first, bool plain, int it, hipStream_t s) {
  dim3 grid(8 * ((v.F * nslots + 7) / 8)), block(kWave * TW);
  const size_t lds = fac_lds_bytes(TW, v.NP, check);
  const int pl = plain ? 1 : 0;
  // x, its anchor, lambda and its anchor stream once per iteration: non-temporal beyond the Infinity Cache
  const int nt = (double)nslots * 4.0 * (double)v.sx * sizeof(float) > 160e6 ? 1 : 0;
  if (init) hipLaunchKernelGGL((fac_x_pass<CPL, false, true, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else if (check)
    hipLaunchKernelGGL((fac_x_pass<CPL, true, false, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else if (first)
    hipLaunchKernelGGL((fac_x_pass<CPL, false, false, true, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else hipLaunchKernelGGL((fac_x_pass<CPL, false, false, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  return hipGetLastError();
}

// waves per workgroup as x_pass (more when few slots iterate), held to 144 KB of LDS
static int fac_tile_waves(const DeviceView &v, int nslots, bool check) {
  int tw = 4;
  while (tw < 16 && (int64_t)nslots * v.F * tw < 4096) tw *= 2;
  if (v.CPL >= 4 && tw > 8) tw = 8;   // (N > 512: 1024-thread workgroups cap a lane at 128 VGPRs, which spill)
  while (tw > 4 && fac_lds_bytes(tw, v.NP, check) > 144 * 1024) tw /= 2;
  return tw;
}

template <int CPL>
static hipError_t launch_fac_cpl(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                                 bool first, bool plain, int it, hipStream_t s) {
  switch (fac_tile_waves(v, nslots, check)) {
    case 4: return launch_fac_tw<CPL, 4>(v, slots, nslots, check, init, first, plain, it, s);
    case 8: return launch_fac_tw<CPL, 8>(v, slots, nslots, check, init, first, plain, it, s);
    case 16: return launch_fac_tw<CPL, 16>(v, slots, nslots, check, init, first, plain, it, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fac_x_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                             bool plain, int it, hipStream_t s) {
  if (fac_lds_bytes(4, v.NP, check) > 144 * 1024) return hipErrorInvalidValue;
  switch (v.CPL) {
    case 1: return launch_fac_cpl<1>(v, slots, nslots, check, init, first, plain, it, s);
    case 2: return launch_fac_cpl<2>(v, slots, nslots, check, init, first, plain, it, s);
    case 4: return launch_fac_cpl<4>(v, slots, nslots, check, init, first, plain, it, s);
    case 8: return launch_fac_cpl<8>(v, slots, nslots, check, init, first, plain, it, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fac_node_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                                bool plain, int it, hipStream_t s) {
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  dim3 grid(v.JB, nslots), block(kNodeThreads);
  if (init) hipLaunchKernelGGL((fac_node_pass<false, true>), grid, block, 0, s, v, slots, fi, pl, it);
  else if (check) hipLaunchKernelGGL((fac_node_pass<true, false>), grid, block, 0, s, v, slots, fi, pl, it);
  else hipLaunchKernelGGL((fac_node_pass<false, false>), grid, block, 0, s, v, slots, fi, pl, it);
  return hipGetLastError();
}

}  // namespace nep
