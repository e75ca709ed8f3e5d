// nep_kernels.hip — gfx950 kernels of one PDHG iteration on a batch of NEPTUNE LP relaxations.
//
// Iteration = one PDHG operator T (diagonally preconditioned; the primal set keeps every routing
// row on its simplex), wrapped in reflected restarted Halpern iterations (r2HPDHG):
//   x̂  = Π_simplex( x̄ − τ (cost_x − Kᵀ_x y) )           x_pass      (HBM-bound)
//   ẑ  = clip( z − τ γ² (cost_z − Kᵀ_z y) )              fj_pass / node_pass / scalar_pass
//   ŷ  = prox( y − σ ρ² K(2·[x̂,ẑ] − [x̄,z]) )             fj_pass / node_pass / scalar_pass
//   w' = λ_k (2·T(w) − w) + (1 − λ_k) w_anchor,  λ_k = (k+1)/(k+2), k = iterations since restart
// ("plain" iterations take w' = T(w): the certificate iteration and the one before it, so the
// certificate's dual is a T output and satisfies the row sign constraints).
// K·[x̂, ẑ] is produced in the same passes that write the iterate (column sums, CPU sums, score
// row); the iterate's activity K w is kept in `kz` (and the anchor's in `kza`, K is linear), so
// K(2ẑ − z) = 2·Kẑ − Kz costs no extra pass.
//
// Reference rows (core/solvers/neptune/utils): C1/C2 constraints_step1.py:5-15 (column sums),
// C3 :18-23, C4 :27-34 (the simplex), C5 :57-65 (CPU), C6/C7 :69-78; step 2 D1-D4
// constraints_step2.py:5-55, score rows :57-88.  Objectives objectives.py:4-63.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>

#include "nep_internal.h"

namespace nep {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_min_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// y' = V − s·clip(V/s, −hi, −lo),  V = y − s·d   (s = σρ²; y ≤ 0 on ≤ rows, ≥ 0 on ≥ rows).
// Evaluated branch-wise so the middle case is an exact 0 (V − s·(V/s) is not) and the sign of y'
// is always right: the Lagrangian bound needs y ≤ 0 on rows without a finite lower bound.
__device__ __forceinline__ double dual_prox(double y, double s, double d, double lo, double hi) {
  const double V = y - s * d;
  const double a = V + s * hi;   // clipped at −hi  (< 0)
  const double b = V + s * lo;   // clipped at −lo  (> 0)
  return a < 0.0 ? a : (b > 0.0 ? b : 0.0);
}
// contribution of a row to the Lagrangian: min over w in [lo,hi] of y·w
__device__ __forceinline__ double row_lagr(double y, double lo, double hi) {
  if (y > 0) return isinf(lo) ? -INFINITY : y * lo;
  if (y < 0) return isinf(hi) ? -INFINITY : y * hi;
  return 0.0;
}
__device__ __forceinline__ double row_viol(double a, double lo, double hi) {
  return fmax(fmax(lo - a, a - hi), 0.0);
}

// ---------------------------------------------------------------------------------------------
// x_pass: one workgroup = one tile (consecutive routing rows of ONE function f) of one LP slot.
// Each wave owns whole rows (N destinations = CPL float4 chunks per lane, 1 KiB per
// wave-instruction), projects each row on its simplex with Michelot's algorithm (wave
// reductions), writes x̄' and accumulates the tile's column sums for the C1/C2/C5 rows.
// ---------------------------------------------------------------------------------------------
template <int CPL, bool CHECK, bool INIT>
__global__ __launch_bounds__(kTileThreads) void x_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                       int plain, int it) {
  constexpr int E = 4 * CPL;
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [2][kTileWaves][NP]
  __shared__ double lds_s[kTileWaves][NTS];
  const int tile = blockIdx.x;
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int NP = v.NP, F = v.F;
  const float tau = INIT ? 0.f : (float)ctrl->tau;
  const bool restart = INIT || (first && ctrl->restart_pending);
  const bool halp = !INIT && !plain;
  float lam = 1.f;
  if (halp) {
    const double ks = (double)(ctrl->ks_base + it);
    lam = (float)((ks + 1.0) / (ks + 2.0));
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  const int f = v.tile_f[tile], row0 = v.tile_row0[tile], nrows = v.tile_nrows[tile];
  float *__restrict__ x = v.x + slot * v.sx;
  float *__restrict__ xa = v.xa + slot * v.sx;
  const uint8_t *__restrict__ mask = v.mask + slot * v.smask + (int64_t)f * NP;
  const float *__restrict__ kty = v.kty + slot * v.skty;
  const float ys = kty[(int64_t)F * NP + NP];

  float kx[E], cy5[E], cp[E];
  bool mk[E];
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j0 = 4 * (lane + kWave * q);
    if (j0 < NP) {
      const float4 a = *reinterpret_cast<const float4 *>(kty + (int64_t)f * NP + j0);
      const float4 b = *reinterpret_cast<const float4 *>(kty + (int64_t)F * NP + j0);
      const float4 c = *reinterpret_cast<const float4 *>(v.cpr + (int64_t)f * NP + j0);
      const uchar4 m = *reinterpret_cast<const uchar4 *>(mask + j0);
      kx[4 * q] = a.x; kx[4 * q + 1] = a.y; kx[4 * q + 2] = a.z; kx[4 * q + 3] = a.w;
      cp[4 * q] = c.x; cp[4 * q + 1] = c.y; cp[4 * q + 2] = c.z; cp[4 * q + 3] = c.w;
      cy5[4 * q] = c.x * b.x; cy5[4 * q + 1] = c.y * b.y; cy5[4 * q + 2] = c.z * b.z; cy5[4 * q + 3] = c.w * b.w;
      mk[4 * q] = m.x; mk[4 * q + 1] = m.y; mk[4 * q + 2] = m.z; mk[4 * q + 3] = m.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) { kx[4 * q + e] = 0.f; cy5[4 * q + e] = 0.f; cp[4 * q + e] = 0.f; mk[4 * q + e] = false; }
    }
  }
  float colS[E], colW[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { colS[e] = 0.f; colW[e] = 0.f; }
  double s_score = 0.0, s_pobj = 0.0, s_lagr = 0.0, s_move = 0.0, s_dist = 0.0, s_empty = 0.0;

  for (int rr = wave; rr < nrows; rr += kTileWaves) {
    const int r = row0 + rr;
    const float m = v.row_m[r], w = v.row_w[r], wobj = v.row_wobj[r], wsc = v.row_wsc[r];
    const int src = v.row_src[r];
    float xv[E], dv[E];
    float *xrow = x + (int64_t)r * NP;
    const bool need_d = src >= 0 && (wobj != 0.f || wsc != 0.f);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), d = make_float4(0.f, 0.f, 0.f, 0.f);
      if (j0 < NP) {
        a = *reinterpret_cast<const float4 *>(xrow + j0);
        if (need_d) d = *reinterpret_cast<const float4 *>(v.D + (int64_t)src * NP + j0);
      }
      xv[4 * q] = a.x; xv[4 * q + 1] = a.y; xv[4 * q + 2] = a.z; xv[4 * q + 3] = a.w;
      dv[4 * q] = d.x; dv[4 * q + 1] = d.y; dv[4 * q + 2] = d.z; dv[4 * q + 3] = d.w;
    }
    // gradient step (reduced cost of x̄[r, j] = cost − Kᵀy)
    float vv[E];
    float s = 0.f;
    int cnt = 0;
    const float gs = wsc * ys;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float g = wobj * dv[e] - (m * kx[e] + w * cy5[e] + gs * dv[e]);
      vv[e] = xv[e] - tau * g;
      if (mk[e]) { s += vv[e]; cnt += 1; }
    }
    if (CHECK) {
      // Lagrangian term of this row: min over the simplex of the reduced cost, in fp64
      double gmin = INFINITY;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (mk[e]) {
          const double g = (double)wobj * dv[e] -
                           ((double)m * kx[e] + (double)w * cy5[e] + (double)wsc * (double)ys * dv[e]);
          gmin = fmin(gmin, g);
        }
      }
      gmin = wave_min_d(gmin);
      if (lane == 0) s_lagr += gmin;
    }
    // Michelot projection onto {x >= 0, sum x = 1} over the allowed destinations
    s = wave_sum(s);
    cnt = wave_sum_i(cnt);
    float theta = INFINITY;
    if (cnt > 0) {
      theta = (s - 1.f) / (float)cnt;
      for (int it = 0; it < 4096; ++it) {
        float s2 = 0.f;
        int c2 = 0;
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (mk[e] && vv[e] > theta) { s2 += vv[e]; c2 += 1; }
        s2 = wave_sum(s2);
        c2 = wave_sum_i(c2);
        if (c2 == cnt || c2 == 0) break;
        cnt = c2;
        theta = (s2 - 1.f) / (float)c2;
      }
    } else if (lane == 0) {
      s_empty += 1.0;
    }
    float xn[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xn[e] = mk[e] ? fmaxf(vv[e] - theta, 0.f) : 0.f;

    float *arow = xa + (int64_t)r * NP;
    // anchor row: needed by the Halpern combination and by the certificate's restart distance
    float xav[E];
    if ((halp || CHECK) && !restart) {
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int j0 = 4 * (lane + kWave * q);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j0 < NP) a = *reinterpret_cast<const float4 *>(arow + j0);
        xav[4 * q] = a.x; xav[4 * q + 1] = a.y; xav[4 * q + 2] = a.z; xav[4 * q + 3] = a.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) xav[e] = INIT ? xn[e] : xv[e];
    }
    if (CHECK && !restart) {
      double dd = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) { const double t = (double)xn[e] - xav[e]; dd += t * t; }
      s_dist += dd;
    }
    float xw[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xw[e] = halp ? lam * (2.f * xn[e] - xv[e]) + (1.f - lam) * xav[e] : xn[e];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      if (j0 < NP) {
        *reinterpret_cast<float4 *>(xrow + j0) = make_float4(xw[4 * q], xw[4 * q + 1], xw[4 * q + 2], xw[4 * q + 3]);
        if (restart)
          *reinterpret_cast<float4 *>(arow + j0) =
              make_float4(xav[4 * q], xav[4 * q + 1], xav[4 * q + 2], xav[4 * q + 3]);
      }
    }
    float sc = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      colS[e] += m * xn[e];
      colW[e] += w * xn[e];
      sc += dv[e] * xn[e];
    }
    s_score += (double)wsc * (double)sc;
    if (CHECK) {
      double po = 0.0, mv = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        po += (double)dv[e] * xn[e];
        const double t = (double)xn[e] - xv[e];
        mv += t * t;
      }
      s_pobj += (double)wobj * po;
      s_move += mv;
    }
  }

  // cross-wave reduction of the tile's column partials
  float *lS = lds, *lW = lds + kTileWaves * NP;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j0 = 4 * (lane + kWave * q);
    if (j0 < NP) {
      *reinterpret_cast<float4 *>(lS + wave * NP + j0) = make_float4(colS[4 * q], colS[4 * q + 1], colS[4 * q + 2], colS[4 * q + 3]);
      *reinterpret_cast<float4 *>(lW + wave * NP + j0) = make_float4(colW[4 * q], colW[4 * q + 1], colW[4 * q + 2], colW[4 * q + 3]);
    }
  }
  double vals[NTS] = {s_score, s_pobj, s_lagr, s_move, s_dist, s_empty};
#pragma unroll
  for (int k = 0; k < NTS; ++k) {
    const double t = wave_sum_d(vals[k]);
    if (lane == 0) lds_s[wave][k] = t;
  }
  __syncthreads();
  float *part = v.part + slot * v.spart + (int64_t)tile * 2 * NP;
  for (int j = threadIdx.x; j < NP; j += kTileThreads) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int wv = 0; wv < kTileWaves; ++wv) { a += lS[wv * NP + j]; b += lW[wv * NP + j]; }
    part[j] = a;
    part[NP + j] = b * v.cpr[(int64_t)f * NP + j];
  }
  if (threadIdx.x < NTS) {
    double t = 0.0;
#pragma unroll
    for (int wv = 0; wv < kTileWaves; ++wv) t += lds_s[wv][threadIdx.x];
    v.tpart[slot * v.stpart + (int64_t)tile * NTS + threadIdx.x] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// fj_pass: one wave per (slot, block of 64 destinations j, block of FPB functions).  Finishes the
// column sums of the tiles of each f, updates c / moved_from / moved_to and the C1/C2/D1/D2 duals,
// writes the packed f32 duals y1+y2 for the x pass, and the per-(f-block, j) partial sums the
// node rows need (memory use, Σ_f c, CPU use).
// ---------------------------------------------------------------------------------------------
struct SmallAcc {
  double lagr = 0, pobj = 0, res = 0, mvz = 0, mvy = 0, dsz = 0, dsy = 0;
};

// Halpern weight of the current iteration for a slot (1 on plain iterations: w' = T(w))
__device__ __forceinline__ double halpern_lambda(const Ctrl *ctrl, bool halp, int it) {
  if (!halp) return 1.0;
  const double ks = (double)(ctrl->ks_base + it);
  return (ks + 1.0) / (ks + 2.0);
}

// Dual half-step of one row.  Returns the new *iterate* y'; `act` is the row activity at the T
// output (K·[x̂, ẑ]).  On a Halpern iteration y' = λ(2ŷ − y) + (1 − λ)y_anchor and the iterate's
// activity kz follows the same combination.
template <bool CHECK, bool INIT>
__device__ __forceinline__ double dual_step(const DeviceView &v, double *y, double *ya, double *kz, double *kza,
                                            int row, double act, double yold, double sigma, bool copy_anchor,
                                            bool halp, double lam, SmallAcc &a) {
  const double lo = v.lo[row], hi = v.hi[row];
  const double kold = kz[row];
  double yanc, kanc;
  if (INIT) {
    yanc = yold;
    kanc = act;
  } else if (copy_anchor) {
    yanc = yold;
    kanc = kold;
  } else {
    yanc = ya[row];
    kanc = kza[row];
  }
  if (copy_anchor) {
    ya[row] = yanc;
    kza[row] = kanc;
  }
  double ynew = yold, knew = act;
  if (!INIT) {
    const double rr = v.rho[row];
    const double yT = dual_prox(yold, sigma * rr * rr, 2.0 * act - kold, lo, hi);
    const double t = (yT - yold) / rr;
    a.mvy += t * t;
    if (CHECK) { const double u = (yT - yanc) / rr; a.dsy += u * u; }
    if (halp) {
      ynew = lam * (2.0 * yT - yold) + (1.0 - lam) * yanc;
      knew = lam * (2.0 * act - kold) + (1.0 - lam) * kanc;
    } else {
      ynew = yT;
    }
    y[row] = ynew;
  }
  kz[row] = knew;
  if (CHECK) {
    a.lagr += row_lagr(yold, lo, hi);
    a.res = fmax(a.res, row_viol(act, lo, hi) / v.rownorm[row]);
  }
  return ynew;
}

// Primal half-step of one small variable.  Stores the new iterate, returns the T output ẑ (the
// value every row activity and the certificate use).
template <bool CHECK>
__device__ __forceinline__ double primal_step(const DeviceView &v, double *zi, double *zia, const double *lb,
                                              const double *ub, int k, double rc, double tau, bool copy_anchor,
                                              bool halp, double lam, SmallAcc &a) {
  const double old = zi[k];
  if (copy_anchor) zia[k] = old;
  const double zanc = copy_anchor ? old : zia[k];
  const double g = v.gam[k];
  const double nz = fmin(fmax(old - tau * g * g * rc, lb[k]), ub[k]);
  zi[k] = halp ? lam * (2.0 * nz - old) + (1.0 - lam) * zanc : nz;
  const double t = (nz - old) / g;
  a.mvz += t * t;
  if (CHECK) {
    const double u = (nz - zanc) / g;
    a.dsz += u * u;
    a.lagr += rc > 0 ? lb[k] * rc : ub[k] * rc;
    a.pobj += v.cost_int[k] * nz;
  }
  return nz;
}

__device__ __forceinline__ void write_bpart(double *bp, const SmallAcc &a, double sumc, double score_n, int lane) {
  double vals[NBS];
  vals[BS_SUMC_NEW] = sumc;
  vals[BS_SCORE_N] = score_n;
  vals[BS_LAGR] = a.lagr;
  vals[BS_POBJ] = a.pobj;
  vals[BS_RES] = a.res;
  vals[BS_MOVE_Z] = a.mvz;
  vals[BS_MOVE_Y] = a.mvy;
  vals[BS_DIST_Z] = a.dsz;
  vals[BS_DIST_Y] = a.dsy;
#pragma unroll
  for (int k = 0; k < NBS; ++k) {
    const double t = (k == BS_RES) ? wave_max_d(vals[k]) : wave_sum_d(vals[k]);
    if (lane == 0) bp[k] = t;
  }
}

template <bool CHECK, bool INIT>
__global__ __launch_bounds__(kWave) void fj_pass(DeviceView v, const int32_t *__restrict__ slots, int first, int plain,
                                                 int it) {
  const int jb = blockIdx.x, fb = blockIdx.y;
  const int slot = slots[blockIdx.z];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int lane = threadIdx.x;
  const int j = jb * kWave + lane;
  const bool valid = j < v.N;
  const int N = v.N, NP = v.NP, F = v.F;
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  const double tau = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool copy_anchor = INIT || (first && ctrl->restart_pending);
  const bool halp = !INIT && !plain;
  const double lam = halpern_lambda(ctrl, halp, it);
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  float *kty = v.kty + slot * v.skty;
  const float *part = v.part + slot * v.spart;
  SmallAcc a;
  double U = 0.0, memc = 0.0, sumc = 0.0;
  const int f0 = fb * v.FPB, f1 = min(F, f0 + v.FPB);
  if (valid) {
    const double y3 = y[dl.o3 + j];
    const double y6 = v.has_n ? y[dl.o6 + j] : 0.0;
    const double y7 = v.has_n ? y[dl.o7 + j] : 0.0;
    const double yD3a = v.step2 ? y[dl.oD3a] : 0.0, yD3b = v.step2 ? y[dl.oD3b] : 0.0;
    const double yD4 = v.step2 ? y[dl.oD4] : 0.0;
    for (int f = f0; f < f1; ++f) {
      double S = 0.0;
      for (int t = v.ftile_ptr[f]; t < v.ftile_ptr[f + 1]; ++t) {
        S += part[(int64_t)t * 2 * NP + j];
        U += part[(int64_t)t * 2 * NP + NP + j];
      }
      const int idx = f * N + j;
      const double y1 = y[dl.o1 + idx], y2 = y[dl.o2 + idx];
      double kty_c = -v.M * y1 - y2 + v.mem_f[f] * y3 + y6 + y7;
      double yd1 = 0.0, yd2 = 0.0;
      if (v.step2) {
        yd1 = y[dl.oD1 + idx];
        yd2 = y[dl.oD2 + idx];
        kty_c += -yd1 + yd2 - yD3a + yD3b + v.sigma4 * yD4;
      }
      const double cn = primal_step<CHECK>(v, zi, zia, lb, ub, il.oc + idx, v.cost_int[il.oc + idx] - kty_c, tau,
                                           copy_anchor, halp, lam, a);
      const double y1n = dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o1 + idx, S - v.M * cn, y1, sigma, copy_anchor,
                                                halp, lam, a);
      const double y2n = dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o2 + idx, S - cn, y2, sigma, copy_anchor, halp,
                                                lam, a);
      if (v.step2) {
        const double mfn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omf + idx, v.cost_int[il.omf + idx] - yd1, tau,
                                              copy_anchor, halp, lam, a);
        const double mtn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omt + idx, v.cost_int[il.omt + idx] - yd2, tau,
                                              copy_anchor, halp, lam, a);
        dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD1 + idx, mfn - cn, yd1, sigma, copy_anchor, halp, lam, a);
        dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD2 + idx, mtn + cn, yd2, sigma, copy_anchor, halp, lam, a);
      }
      memc += v.mem_f[f] * cn;
      sumc += cn;
      kty[(int64_t)f * NP + j] = (float)(y1n + y2n);
    }
    double *np_ = v.npart + slot * v.snpart + (int64_t)fb * 3 * NP;
    np_[j] = memc;
    np_[NP + j] = sumc;
    np_[2 * NP + j] = U;
  }
  write_bpart(v.bpart + slot * v.sbpart + ((int64_t)fb * v.JB + jb) * NBS, a, valid ? sumc : 0.0, 0.0, lane);
}

// node_pass: one wave per (slot, block of 64 nodes j): rows C3 (memory), C5 (CPU), n, C6/C7.
template <bool CHECK, bool INIT>
__global__ __launch_bounds__(kWave) void node_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                   int plain, int it) {
  const int jb = blockIdx.x;
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int lane = threadIdx.x;
  const int j = jb * kWave + lane;
  const bool valid = j < v.N;
  const int NP = v.NP, F = v.F;
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  const double tau = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool copy_anchor = INIT || (first && ctrl->restart_pending);
  const bool halp = !INIT && !plain;
  const double lam = halpern_lambda(ctrl, halp, it);
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  float *kty = v.kty + slot * v.skty;
  SmallAcc a;
  double score_n = 0.0;
  if (valid) {
    double memc = 0.0, sumc = 0.0, U = 0.0;
    const double *np_ = v.npart + slot * v.snpart;
    for (int fb = 0; fb < v.FB; ++fb) {
      memc += np_[(int64_t)fb * 3 * NP + j];
      sumc += np_[(int64_t)fb * 3 * NP + NP + j];
      U += np_[(int64_t)fb * 3 * NP + 2 * NP + j];
    }
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o3 + j, memc, y[dl.o3 + j], sigma, copy_anchor, halp, lam, a);
    const double y5n = dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o5 + j, U, y[dl.o5 + j], sigma, copy_anchor, halp,
                                              lam, a);
    kty[(int64_t)F * NP + j] = (float)y5n;
    if (v.has_n) {
      const double y6 = y[dl.o6 + j], y7 = y[dl.o7 + j];
      const double yS = v.step2 ? y[dl.oS] : 0.0;
      const double kty_n = -v.M * y6 - y7 + v.score_n_coef * yS;
      const double nn = primal_step<CHECK>(v, zi, zia, lb, ub, il.on + j, v.cost_int[il.on + j] - kty_n, tau,
                                           copy_anchor, halp, lam, a);
      dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o6 + j, sumc - v.M * nn, y6, sigma, copy_anchor, halp, lam, a);
      dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o7 + j, sumc - nn, y7, sigma, copy_anchor, halp, lam, a);
      score_n = v.score_n_coef * nn;
    }
  }
  write_bpart(v.bpart + slot * v.sbpart + ((int64_t)v.FB * v.JB + jb) * NBS, a, 0.0, score_n, lane);
}

// ---------------------------------------------------------------------------------------------
// scalar_pass: one workgroup per slot.  Step-2 scalar rows (D3a, D3b, D4, score) and the
// integer-bounded a / d variables; at check iterations the certificate (primal objective,
// Lagrangian bound, residuals), status, restarts and the primal-weight update.
// ---------------------------------------------------------------------------------------------
template <bool CHECK, bool INIT>
__global__ __launch_bounds__(256) void scalar_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                   int plain, int it, int iters_done, int block_len) {
  __shared__ double red[256];
  __shared__ double tot[NTS + NBS];
  const int slot = slots[blockIdx.x];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int tid = threadIdx.x;
  const double *tp = v.tpart + slot * v.stpart;
  const double *bp = v.bpart + slot * v.sbpart;
  const int nb = v.FB * v.JB + v.JB;
  // deterministic block reductions (fixed order per thread, fixed tree)
  for (int k = 0; k < NTS + NBS; ++k) {
    const bool is_max = (k == NTS + BS_RES);
    double acc = 0.0;
    if (k < NTS) {
      for (int t = tid; t < v.T; t += 256) acc += tp[(int64_t)t * NTS + k];
    } else {
      for (int t = tid; t < nb; t += 256) {
        const double u = bp[(int64_t)t * NBS + (k - NTS)];
        acc = is_max ? fmax(acc, u) : acc + u;
      }
    }
    red[tid] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) red[tid] = is_max ? fmax(red[tid], red[tid + s]) : red[tid] + red[tid + s];
      __syncthreads();
    }
    if (tid == 0) tot[k] = red[0];
    __syncthreads();
  }
  if (tid != 0) return;

  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  const double tau = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool copy_anchor = INIT || (first && ctrl->restart_pending);
  const bool halp = !INIT && !plain;
  const double lam = halpern_lambda(ctrl, halp, it);
  SmallAcc a;
  a.lagr = tot[TS_LAGR] + tot[NTS + BS_LAGR];
  a.pobj = tot[TS_POBJ] + tot[NTS + BS_POBJ];
  a.res = tot[NTS + BS_RES];
  a.mvz = tot[TS_MOVE] + tot[NTS + BS_MOVE_Z];
  a.mvy = tot[NTS + BS_MOVE_Y];
  a.dsz = tot[TS_DIST] + tot[NTS + BS_DIST_Z];
  a.dsy = tot[NTS + BS_DIST_Y];

  if (v.step2) {
    const double sumc = tot[NTS + BS_SUMC_NEW];
    const double score = tot[TS_SCORE] + tot[NTS + BS_SCORE_N];
    const double yD3a = y[dl.oD3a], yD3b = y[dl.oD3b], yD4 = y[dl.oD4], yS = y[dl.oS];
    // allocated (a): D3a coef -1, D4 coef +1 ; deallocated (d): D3b coef -1, D4 coef +1
    const double an = primal_step<CHECK>(v, zi, zia, lb, ub, il.oa, v.cost_int[il.oa] - (-yD3a + yD4), tau,
                                         copy_anchor, halp, lam, a);
    const double dn = primal_step<CHECK>(v, zi, zia, lb, ub, il.od, v.cost_int[il.od] - (-yD3b + yD4), tau,
                                         copy_anchor, halp, lam, a);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD3a, -sumc - an, yD3a, sigma, copy_anchor, halp, lam, a);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD3b, sumc - dn, yD3b, sigma, copy_anchor, halp, lam, a);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD4, dn + an + v.sigma4 * sumc, yD4, sigma, copy_anchor, halp, lam,
                           a);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oS, score, yS, sigma, copy_anchor, halp, lam, a);
    float *kty = v.kty + slot * v.skty;
    kty[(int64_t)v.F * v.NP + v.NP] = (float)y[dl.oS];
  }
  if (INIT) {
    ctrl->restart_pending = 0;
    ctrl->k = 0;
    ctrl->k_since_restart = 0;
    ctrl->ks_base = -block_len;   // the first certificate iteration brings it to 0
    ctrl->last_restart_fpr = -1.0;
    ctrl->prev_fpr = INFINITY;
    return;
  }
  if (!CHECK) return;

  ctrl->k += iters_done;
  ctrl->k_since_restart += iters_done;
  ctrl->restart_pending = 0;
  if (tot[TS_EMPTY] > 0) { ctrl->status = 2; ctrl->active = 0; return; }
  const double lagr = a.lagr, pobj = a.pobj, res = a.res;
  const double gap = pobj - lagr;
  ctrl->pobj = pobj;
  ctrl->lagr = lagr;
  if (lagr > ctrl->best_lagr) ctrl->best_lagr = lagr;
  ctrl->pres = res;
  ctrl->gap = gap;
  if (isfinite(lagr) && res <= v.tol && gap <= v.tol * fmax(1.0, fabs(lagr))) {
    ctrl->status = 0; ctrl->active = 0; return;
  }
  if (ctrl->best_lagr > v.cutoff) { ctrl->status = 3; ctrl->active = 0; return; }
  if (ctrl->k >= v.max_iters) { ctrl->status = 1; ctrl->active = 0; return; }
  if (!isfinite(pobj) || !isfinite(a.mvz) || !isfinite(a.mvy)) { ctrl->status = 4; ctrl->active = 0; return; }

  // restart test on the fixed-point residual of the last iteration (ω-weighted norm)
  const double w = ctrl->omega;
  const double fpr = sqrt(w * a.mvz + a.mvy / w);
  if (ctrl->last_restart_fpr < 0) ctrl->last_restart_fpr = fpr;
  const bool restart = (fpr <= 0.2 * ctrl->last_restart_fpr) ||
                       (fpr <= 0.8 * ctrl->last_restart_fpr && fpr > ctrl->prev_fpr) ||
                       (ctrl->k_since_restart >= 0.36 * ctrl->k);
  ctrl->prev_fpr = fpr;
  if (restart) {
    const double dz = sqrt(a.dsz), dy = sqrt(a.dsy);
    if (dz > 1e-10 && dy > 1e-10) {
      double nw = exp(0.5 * log(dy / dz) + 0.5 * log(w));
      nw = fmin(fmax(nw, ctrl->omega_lo), ctrl->omega_hi);
      ctrl->omega = nw;
      ctrl->tau = ctrl->eta / nw;
      ctrl->sigma = ctrl->eta * nw;
    }
    ctrl->restart_pending = 1;   // consumed by the passes of the block's next iteration (it == 1)
    ctrl->k_since_restart = 0;
    ctrl->ks_base = -1;          // Halpern counter: 0 at the iteration that sets the anchor
    ctrl->last_restart_fpr = fpr;
    ctrl->prev_fpr = INFINITY;
  } else {
    ctrl->ks_base += block_len;
  }
}

// cold / warm initialisation of a slot (x̄ ← 0 for cold; the init passes project it)
__global__ void init_slot(DeviceView v, const int32_t *__restrict__ slots, int warm, double eta, double omega0) {
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double *zi = v.zi + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  if (!warm) {
    float *x = v.x + slot * v.sx;
    for (int64_t i = tid; i < (int64_t)v.R * v.NP; i += stride) x[i] = 0.f;
    double *y = v.y + slot * v.sdual;
    for (int64_t i = tid; i < v.dl.n_dual; i += stride) y[i] = 0.0;
    float *kty = v.kty + slot * v.skty;
    for (int64_t i = tid; i < v.skty; i += stride) kty[i] = 0.f;
  }
  for (int64_t i = tid; i < v.il.n_int; i += stride) {
    const double z0 = warm ? zi[i] : 0.0;
    zi[i] = fmin(fmax(z0, lb[i]), ub[i]);
  }
  if (tid == 0) {
    if (!warm) ctrl->omega = omega0;
    ctrl->eta = eta;
    ctrl->omega_lo = omega0 * 1e-5;
    ctrl->omega_hi = omega0 * 1e5;
    ctrl->tau = eta / ctrl->omega;
    ctrl->sigma = eta * ctrl->omega;
    ctrl->status = 1;
    ctrl->active = 1;
    ctrl->restart_pending = 1;
    ctrl->best_lagr = -INFINITY;
    ctrl->pobj = ctrl->lagr = ctrl->pres = ctrl->gap = NAN;
  }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int CPL>
static hipError_t launch_x_cpl(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                               bool first, bool plain, int it, hipStream_t s) {
  dim3 grid(v.T, nslots), block(kTileThreads);
  const size_t lds = (size_t)2 * kTileWaves * v.NP * sizeof(float);
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  if (init) hipLaunchKernelGGL((x_pass<CPL, false, true>), grid, block, lds, s, v, slots, fi, pl, it);
  else if (check) hipLaunchKernelGGL((x_pass<CPL, true, false>), grid, block, lds, s, v, slots, fi, pl, it);
  else hipLaunchKernelGGL((x_pass<CPL, false, false>), grid, block, lds, s, v, slots, fi, pl, it);
  return hipGetLastError();
}

hipError_t launch_x_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                         bool plain, int it, hipStream_t s) {
  switch (v.CPL) {
    case 1: return launch_x_cpl<1>(v, slots, nslots, check, init, first, plain, it, s);
    case 2: return launch_x_cpl<2>(v, slots, nslots, check, init, first, plain, it, s);
    case 4: return launch_x_cpl<4>(v, slots, nslots, check, init, first, plain, it, s);
    case 8: return launch_x_cpl<8>(v, slots, nslots, check, init, first, plain, it, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_small_passes(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                               bool first, bool plain, int it, hipStream_t s) {
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  dim3 g1(v.JB, v.FB, nslots), g2(v.JB, nslots), block(kWave);
  if (init) {
    hipLaunchKernelGGL((fj_pass<false, true>), g1, block, 0, s, v, slots, fi, pl, it);
    hipLaunchKernelGGL((node_pass<false, true>), g2, block, 0, s, v, slots, fi, pl, it);
  } else if (check) {
    hipLaunchKernelGGL((fj_pass<true, false>), g1, block, 0, s, v, slots, fi, pl, it);
    hipLaunchKernelGGL((node_pass<true, false>), g2, block, 0, s, v, slots, fi, pl, it);
  } else {
    hipLaunchKernelGGL((fj_pass<false, false>), g1, block, 0, s, v, slots, fi, pl, it);
    hipLaunchKernelGGL((node_pass<false, false>), g2, block, 0, s, v, slots, fi, pl, it);
  }
  return hipGetLastError();
}

hipError_t launch_scalar_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                              bool first, bool plain, int it, int iters_done, int block_len, hipStream_t s) {
  dim3 grid(nslots), block(256);
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  if (init)
    hipLaunchKernelGGL((scalar_pass<false, true>), grid, block, 0, s, v, slots, fi, pl, it, iters_done, block_len);
  else if (check)
    hipLaunchKernelGGL((scalar_pass<true, false>), grid, block, 0, s, v, slots, fi, pl, it, iters_done, block_len);
  else
    hipLaunchKernelGGL((scalar_pass<false, false>), grid, block, 0, s, v, slots, fi, pl, it, iters_done, block_len);
  return hipGetLastError();
}

hipError_t launch_init_slot(const DeviceView &v, const int32_t *slots, int nslots, bool warm, double eta,
                            double omega0, hipStream_t s) {
  dim3 grid(256, nslots), block(256);
  hipLaunchKernelGGL(init_slot, grid, block, 0, s, v, slots, warm ? 1 : 0, eta, omega0);
  return hipGetLastError();
}

}  // namespace nep
