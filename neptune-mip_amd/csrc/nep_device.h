// nep_device.h — device helpers shared by the PDHG passes of the reference model (nep_kernels.hip) and of the
// facility relaxation (nep_fac.hip): wave reductions, dual proximal step, Lagrangian row terms, the step-2
// disruption block and the big-M dual repair, the per-row / per-variable PDHG half-steps and the routing-row
// loads.  Included by .hip translation units only.
#pragma once
#include <hip/hip_runtime.h>
#include <cfloat>
#include <algorithm>
#include <cmath>

#include "nep_internal.h"

namespace nep {

// ---------------------------------------------------------------------------------------------
// wave reductions
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Wave-uniform f32 sum: DPP butterfly inside each 16-lane row (quad_perm [1,0,3,2], quad_perm
// [2,3,0,1], row_ror:4, row_ror:8 — every lane of a row then holds the row sum), then the four
// row sums read as scalars.  No LDS-crossbar (ds_bpermute) round trips; every lane gets the same
// value in the same summation order.
__device__ __forceinline__ float wave_sum_u(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x124>(v);
  v += dpp_f<0x128>(v);
  return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}
__device__ __forceinline__ float wave_max_u(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x128>(v));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
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

struct SmallAcc {
  double lagr = 0, pobj = 0, res = 0, mvz = 0, mvy = 0, dsz = 0, dsy = 0;
  double lagrD = 0;   // Lagrangian terms of the step-2 disruption block (dblk calls)
  double lagrR = 0;   // certificate: Lagrangian terms at the repaired duals (DESIGN.md §4 "Dual repair")
  double lagr0 = 0;   // certificate: every Lagrangian term with the objective off (DESIGN.md §4 "Infeasibility")
};

// ---------------------------------------------------------------------------------------------
// Step-2 disruption block kept exact in the bound (DESIGN.md §4 "Disruption block").  The rows
// D1/D2 (moved_from/to vs c and old), D3a/D3b/D4 (allocated / deallocated vs sum c) carry duals
// against costs F*N, F*N +- 1: fp32-level relative noise on them moves the plain Lagrangian by ~1e-5
// (tools/probes/dblock_probe.py), more than the 1e-6 certificate allows.  Instead of dualising them, the
// bound minimises the block exactly: sum c is relaxed to a free T priced by lambda, each (f, j) takes
// min over (c, mf, mt) of (r' - lambda) c + cmf mf + cmt mt on its box and D1/D2 (a piecewise-linear
// function of c: its minimum is at an end or a kink), and G(lambda) = min over (a, d, T) of
// ca a + cd d + lambda T on the boxes and D3a/D3b/D4 (a 3-variable LP: the best vertex).  For every
// lambda that is a valid lower bound; kNLam candidates are evaluated in the same pass: the PDHG's own
// price of sum c and the slopes +-ca, +-cd, 0 that the optimal price takes unless a D3 cap binds.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void dblock_lambdas(const DeviceView &v, const double *y, double (&lam)[kNLam]) {
  const double ca = v.cost_int[v.il.oa], cd = v.cost_int[v.il.od];
  lam[0] = -y[v.dl.oD3a] + y[v.dl.oD3b] + v.sigma4 * y[v.dl.oD4];
  lam[1] = -cd;
  lam[2] = ca;
  lam[3] = -ca;
  lam[4] = cd;
  lam[5] = 0.0;
}

// min over c of (r - lam) c + cmf max(lmf, c - old) + cmt max(lmt, old - c), c in [clo, chi]
__device__ __forceinline__ double dblock_item(double r, double lam, double old, double cmf, double lmf, double cmt,
                                              double lmt, double clo, double chi) {
  if (clo > chi) return INFINITY;
  const double pts[4] = {clo, chi, fmin(fmax(old + lmf, clo), chi), fmin(fmax(old - lmt, clo), chi)};
  double best = INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double c = pts[q];
    best = fmin(best, (r - lam) * c + cmf * fmax(lmf, c - old) + cmt * fmax(lmt, old - c));
  }
  return best;
}

// ---------------------------------------------------------------------------------------------
// Dual repair of the big-M row pairs at certificate iterations (DESIGN.md §4 "Dual repair").  C1/C2
// (S - M c <= 0, S - c >= -eps) enter c's reduced cost as M*y1 + y2 and the routing columns as
// y1 + y2 =: s; C6/C7 enter n's as M*y6 + y7 and c's as y6 + y7 =: t.  At an LP optimum an interior
// c (e.g. c = S / M) has reduced cost exactly 0, so a dual error d in s moves the Lagrangian by M*d
// (the box of c has width 1); and a column price the PDHG has not resolved at the 1e-6 level (the
// 1/M price of routing flow to a destination that is not the old placement) drops that whole part
// of the objective from the bound (tools/probes/dual_repair_probe.py).  The repair re-prices
// each pair from the iterate's own c (complementary slackness, as a crossover would):
//   * c inside a linear piece of its (disruption-)cost: the price that makes that piece's slope 0;
//   * c at 0 = its lower end: the lowest price keeping c = 0 a minimiser (lowering s never lowers the
//     routing rows' terms, and c's term stays 0);
//   * otherwise (c at an upper end / kink): the price among the breakpoints (s0 first) that
//     maximises the pair's own terms, with the routing rows' change bounded pessimistically (raising
//     s by D lowers every routing row of f by at most its weight times D, N in all).
// s is split back as y1 = min(0, s), y2 = max(0, s); t alike from n.  Any sign-feasible dual gives a
// valid bound: the certificate takes the better of the plain and the repaired one.
// ---------------------------------------------------------------------------------------------
constexpr double kRepairTol = 1e-7;   // an iterate within this of a box end / kink sits on it
__device__ __forceinline__ double price_rc(double b, double s, double M) { return b + M * fmin(s, 0.0) + fmax(s, 0.0); }
__device__ __forceinline__ double price_at(double b, double target, double M) {
  const double d = target - b;   // the s with price_rc(b, s) == target
  return d < 0.0 ? d / M : d;
}
// a (c or n) on its box [lb, ub] with reduced cost price_rc(b, s); z its iterate
__device__ __forceinline__ double repair_box(double b, double s0, double z, double lb, double ub, double M,
                                             double eps, double K) {
  if (z > lb + kRepairTol && z < ub - kRepairTol) return price_at(b, 0.0, M);   // interior: reduced cost 0
  if (z <= lb + kRepairTol && lb == 0.0) return price_at(b, 0.0, M);           // at 0: lowest price keeping it
  const double cand[4] = {s0, 0.0, price_at(b, 0.0, M), -b};
  double best = -INFINITY, sb = s0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double s = cand[q], rc = price_rc(b, s, M);
    const double val = fmin(rc * lb, rc * ub) - eps * fmax(s, 0.0) - K * fmax(s - s0, 0.0);
    if (val > best) { best = val; sb = s; }
  }
  return sb;
}
// step 2: c with its disruption block (dblock_item) at the price lam of sum c; z its iterate.  The
// block's cost in c has slopes (r - lam) - cmt / (r - lam) / (r - lam) + cmf on the pieces split at
// the kinks old - lmt and old + lmf.
__device__ __forceinline__ double repair_dblock(double b, double s0, double z, double lam, double old, double cmf,
                                                double lmf, double cmt, double lmt, double clo, double chi, double M,
                                                double eps, double K) {
  const double k1 = old - lmt, k2 = old + lmf, t = kRepairTol;
  const bool at_k = fabs(z - k1) <= t || fabs(z - k2) <= t;
  const double piece = z < k1 ? -cmt : (z > k2 ? cmf : 0.0);          // slope constant of z's piece
  if (z > clo + t && z < chi - t && !at_k) return price_at(b, lam - piece, M);
  if (z <= clo + t && clo == 0.0 && clo < chi) {
    // lowest price keeping c = 0 a minimiser: the slope right of 0 is >= 0
    const double right = (0.0 >= k2 - t) ? cmf : ((0.0 >= k1 - t) ? 0.0 : -cmt);
    return price_at(b, lam - right, M);
  }
  const double cand[5] = {s0, 0.0, price_at(b, lam + cmt, M), price_at(b, lam, M), price_at(b, lam - cmf, M)};
  double best = -INFINITY, sb = s0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const double s = cand[q];
    const double val = dblock_item(price_rc(b, s, M), lam, old, cmf, lmf, cmt, lmt, clo, chi) - eps * fmax(s, 0.0) -
                       K * fmax(s - s0, 0.0);
    if (val > best) { best = val; sb = s; }
  }
  return sb;
}
// the price of sum c the repair aims at: the PDHG's own (lam[0]) snapped to a fixed candidate price
// (+-ca, +-cd, 0) when within 1e-6 of it — the optimal price is usually one of them exactly, and
// T = sum c ranges over [0, F N], so a price off by d costs up to F N d
__device__ __forceinline__ double repair_lambda(const double (&lam)[kNLam]) {
#pragma unroll
  for (int q = 1; q < kNLam; ++q)
    if (fabs(lam[0] - lam[q]) <= 1e-6 * fmax(1.0, fabs(lam[q]))) return lam[q];
  return lam[0];
}
// n[j]'s reduced cost without C6/C7 (its cost and the step-2 score row); pre-update duals
__device__ __forceinline__ double node_base(const DeviceView &v, const double *y, int j) {
  return v.cost_int[v.il.on + j] - v.score_n_coef * (v.step2 ? y[v.dl.oS] : 0.0);
}
// node j's repaired C6/C7 price t* (n's own terms; raising t lowers each c[f, j]'s term by at most its
// width: F in all); n: the iterate
__device__ __forceinline__ double repair_node(const DeviceView &v, double t0, double b, double n, double lbn,
                                              double ubn) {
  return repair_box(b, t0, n, lbn, ubn, v.M, v.eps, (double)v.F);
}
__device__ __forceinline__ double repaired_node_price(const DeviceView &v, int slot, int j) {
  const double *y = v.y + slot * v.sdual, *zi = v.zi + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  const int k = v.il.on + j;
  return repair_node(v, y[v.dl.o6 + j] + y[v.dl.o7 + j], node_base(v, y, j), zi[k], lb[k], ub[k]);
}
// c[f, j]'s reduced cost without C1/C2 (and without the step-2 D rows, which dblock_item keeps exact),
// at node j's repaired C6/C7 price
__device__ __forceinline__ double repaired_c_base(const DeviceView &v, int slot, int f, int j) {
  const double *y = v.y + slot * v.sdual;
  double b = v.cost_int[v.il.oc + f * v.N + j] - v.mem_f[f] * y[v.dl.o3 + j];
  if (v.has_n) b -= repaired_node_price(v, slot, j);
  return b;
}
// Step 2, reduced disruption block (DeviceView::dred): c[f, j]'s own cost once moved_from /
// moved_to / allocated / deallocated take their LP optimum given c — integral moved bounds: old = 0 ->
// mf = max(lmf, c) (w c if lmf = 0, else the constant w), mt = lmt; old = 1 -> mt = max(lmt, 1 - c)
// (w (1 - c) if lmt = 0, else w), mf = lmf — plus sT per unit of sum c (allocated / deallocated, dred_interval).
// cconst: the (f, j)'s constant part of that cost (the objective and the bound add it).
__device__ __forceinline__ double dred_cost(const DeviceView &v, const double *lb, int idx, double &cconst) {
  const double old = -v.lo[v.dl.oD1 + idx], w = v.w_dis;
  const double lmf = lb[v.il.omf + idx], lmt = lb[v.il.omt + idx];
  double c;
  if (old < 0.5) {
    c = lmf < 0.5 ? w : 0.0;
    cconst = w * (lmf + lmt);
  } else {
    c = lmt < 0.5 ? -w : 0.0;
    cconst = w * (lmf + 1.0);
  }
  return c + v.sT;
}
// the row sum c in [L, U] of the reduced block (D4's dual): L / U from the slot's allocated / deallocated box
__device__ __forceinline__ void dred_bounds(const DeviceView &v, const double *lb, const double *ub, double &L,
                                            double &U) {
  double tlo, thi;
  dred_interval(v.sigma4, lb[v.il.oa], ub[v.il.oa], lb[v.il.od], ub[v.il.od], tlo, thi);
  L = v.sum_old + tlo;
  U = v.sum_old + thi;
}

// the repaired column price s*[f, j] = y1 + y2 of C1/C2 (lam: the step-2 price of sum c); pre-update
// duals and iterate (x_pass's certificate launch, before it updates them)
__device__ __forceinline__ double repaired_col_price(const DeviceView &v, int slot, int f, int j, double lam) {
  const double *y = v.y + slot * v.sdual, *zi = v.zi + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  const IntLayout &il = v.il;
  const int idx = f * v.N + j;
  const double b = repaired_c_base(v, slot, f, j), s0 = y[v.dl.o1 + idx] + y[v.dl.o2 + idx];
  const double z = zi[il.oc + idx];
  if (!v.step2) return repair_box(b, s0, z, lb[il.oc + idx], ub[il.oc + idx], v.M, v.eps, (double)v.N);
  if (v.dred) {   // c's own (linear) cost and the row sum c's dual, on c's box (moved bounds propagated)
    double cc;
    const double bd = b + dred_cost(v, lb, idx, cc) - y[v.dl.oD4];
    return repair_box(bd, s0, z, lb[il.oc + idx], ub[il.oc + idx], v.M, v.eps, (double)v.N);
  }
  const double old = -v.lo[v.dl.oD1 + idx];
  const double clo = fmax(lb[il.oc + idx], old - ub[il.omt + idx]), chi = fmin(ub[il.oc + idx], old + ub[il.omf + idx]);
  return repair_dblock(b, s0, z, lam, old, v.cost_int[il.omf + idx], lb[il.omf + idx], v.cost_int[il.omt + idx],
                       lb[il.omt + idx], clo, chi, v.M, v.eps, (double)v.N);
}

// Operands of one dual row / one small variable, loaded ahead of their update (node_pass issues
// every load of its rows at kernel start, so they overlap the partial sums instead of forming a
// load -> store -> load chain through possibly aliasing pointers).
struct DPre {
  double y, lo, hi, rho, kz, ya, kza;
};
struct ZPre {
  double z, za, lb, ub, gam, cost;
};
template <bool INIT>
__device__ __forceinline__ DPre dual_pre(const DeviceView &v, const double *y, const double *ya, const double *kz,
                                         const double *kza, int row, bool copy_anchor) {
  DPre p;
  p.y = y[row];
  p.lo = v.lo[row];
  p.hi = v.hi[row];
  p.rho = v.rho[row];
  p.kz = kz[row];
  p.ya = (INIT || copy_anchor) ? 0.0 : ya[row];
  p.kza = (INIT || copy_anchor) ? 0.0 : kza[row];
  return p;
}
__device__ __forceinline__ ZPre primal_pre(const DeviceView &v, const double *zi, const double *zia, const double *lb,
                                           const double *ub, int k, bool copy_anchor) {
  ZPre p;
  p.z = zi[k];
  p.za = copy_anchor ? 0.0 : zia[k];
  p.lb = lb[k];
  p.ub = ub[k];
  p.gam = v.gam[k];
  p.cost = v.cost_int[k];
  return p;
}

// Dual half-step of one row.  Returns the new *iterate* y'; `act` is the row activity at the T
// output (K·[x̂, ẑ]).  On a Halpern iteration y' = λ(2ŷ − y) + (1 − λ)y_anchor and the iterate's
// activity kz follows the same combination.
template <bool CHECK, bool INIT>
__device__ __forceinline__ double dual_step_p(double *y, double *ya, double *kz, double *kza, int row, double act,
                                              const DPre &p, double sigma, bool copy_anchor, bool halp, double lam,
                                              SmallAcc &a, bool dblk = false) {
  const double lo = p.lo, hi = p.hi, yold = p.y;
  const double kold = p.kz;
  double yanc, kanc;
  if (INIT) {
    yanc = yold;
    kanc = act;
  } else if (copy_anchor) {
    yanc = yold;
    kanc = kold;
  } else {
    yanc = p.ya;
    kanc = p.kza;
  }
  if (copy_anchor) {
    ya[row] = yanc;
    kza[row] = kanc;
  }
  double ynew = yold, knew = act;
  if (!INIT) {
    const double rr = p.rho;
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
    const double t = row_lagr(yold, lo, hi);
    (dblk ? a.lagrD : a.lagr) += t;
    a.lagr0 += t;
  }
  return ynew;
}
template <bool CHECK, bool INIT>
__device__ __forceinline__ double dual_step(const DeviceView &v, double *y, double *ya, double *kz, double *kza,
                                            int row, double act, double yold, double sigma, bool copy_anchor,
                                            bool halp, double lam, SmallAcc &a, bool dblk = false) {
  DPre p = dual_pre<INIT>(v, y, ya, kz, kza, row, copy_anchor);
  p.y = yold;
  return dual_step_p<CHECK, INIT>(y, ya, kz, kza, row, act, p, sigma, copy_anchor, halp, lam, a, dblk);
}

// Dual half-step of a row whose reflected activity K(2ŵ - w) the caller forms itself from values it
// already holds (C1/C2: the reflected column sum of x and 2ĉ - c; D1/D2: the small variables), so the
// per-(f, j) activities kz / kza are neither read nor written (48 B per (f, j) and LP-iteration).
template <bool CHECK, bool INIT>
__device__ __forceinline__ double dual_step_refl(const DeviceView &v, double *y, double *ya, int row, double refl,
                                                 double yold, double sigma, bool copy_anchor, bool halp, double lam,
                                                 SmallAcc &a, bool dblk = false) {
  const double lo = v.lo[row], hi = v.hi[row];
  double ynew = yold;
  if (!INIT) {
    const double rr = v.rho[row];
    const double yanc = copy_anchor ? yold : ya[row];
    if (copy_anchor) ya[row] = yanc;
    const double yT = dual_prox(yold, sigma * rr * rr, refl, lo, hi);
    const double t = (yT - yold) / rr;
    a.mvy += t * t;
    if (CHECK) { const double u = (yT - yanc) / rr; a.dsy += u * u; }
    ynew = halp ? lam * (2.0 * yT - yold) + (1.0 - lam) * yanc : yT;
    y[row] = ynew;
  } else {
    ya[row] = yold;
  }
  if (CHECK) {
    const double t = row_lagr(yold, lo, hi);
    (dblk ? a.lagrD : a.lagr) += t;
    a.lagr0 += t;
  }
  return ynew;
}

// Primal half-step of one small variable.  Stores the new iterate, returns the T output ẑ (the
// value every row activity and the certificate use).  rc = cost - Kᵀy.
template <bool CHECK>
__device__ __forceinline__ double primal_step_p(double *zi, double *zia, int k, double rc, const ZPre &p, double tau,
                                                bool copy_anchor, bool halp, double lam, SmallAcc &a,
                                                bool dblk = false) {
  const double old = p.z;
  if (copy_anchor) zia[k] = old;
  const double zanc = copy_anchor ? old : p.za;
  const double g = p.gam;
  const double nz = fmin(fmax(old - tau * g * g * rc, p.lb), p.ub);
  zi[k] = halp ? lam * (2.0 * nz - old) + (1.0 - lam) * zanc : nz;
  const double t = (nz - old) / g;
  a.mvz += t * t;
  if (CHECK) {
    const double u = (nz - zanc) / g;
    a.dsz += u * u;
    (dblk ? a.lagrD : a.lagr) += rc > 0 ? p.lb * rc : p.ub * rc;
    const double rc0 = rc - p.cost;   // (rc carries the cost except while polishing, when lagr0 is unused)
    a.lagr0 += rc0 > 0 ? p.lb * rc0 : p.ub * rc0;
  }
  return nz;
}
template <bool CHECK>
__device__ __forceinline__ double primal_step(const DeviceView &v, double *zi, double *zia, const double *lb,
                                              const double *ub, int k, double rc, double tau, bool copy_anchor,
                                              bool halp, double lam, SmallAcc &a, bool dblk = false) {
  const ZPre p = primal_pre(v, zi, zia, lb, ub, k, copy_anchor);
  return primal_step_p<CHECK>(zi, zia, k, rc, p, tau, copy_anchor, halp, lam, a, dblk);
}

// Halpern weight of the current iteration for a slot (1 on plain iterations: w' = T(w))
__device__ __forceinline__ double halpern_lambda(const Ctrl *ctrl, bool halp, int it) {
  if (!halp) return 1.0;
  const double ks = (double)(ctrl->ks_base + it);
  return (ks + 1.0) / (ks + 2.0);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
// the routing-state streams (x, anchor): read and written once per iteration, so non-temporal
// (NEP_NT): they then do not push the delay rows D[src, :] — re-read by every row of a function
// and by every LP slot — out of the XCD's L2
// `nt` is chosen per launch by the host (launch_x_tw): only when the iterating slots' routing state
// exceeds what the 256 MiB Infinity Cache can keep between iterations — a lone root LP (55 MB of x +
// anchor at 512x256) streams from the Infinity Cache with default-policy loads, 32 slots (1.8 GB)
// cannot.
__device__ __forceinline__ f32x4 ld_x4(const float *p, bool nt) {
  if (NEP_NT && nt) return __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
  return *reinterpret_cast<const f32x4 *>(p);
}
__device__ __forceinline__ void st_x4(float *p, f32x4 v, bool nt) {
  if (NEP_NT && nt) __builtin_nontemporal_store(v, reinterpret_cast<f32x4 *>(p));
  else *reinterpret_cast<f32x4 *>(p) = v;
}

// one routing row's operands: x̄ row, delay row D[src, :] (if the row has delay-weighted
// coefficients) and the dense anchor row (if needed and the row's anchor is held dense)
template <int CPL>
__device__ __forceinline__ void load_row(const float *__restrict__ xrow, const float *__restrict__ drow,
                                         const float *__restrict__ arow, bool nd, bool na, bool nt, int lane,
                                         int NP, float (&xo)[4 * CPL], float (&dout)[4 * CPL], float (&ao)[4 * CPL]) {
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j0 = 4 * (lane + kWave * q);
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, an = a;
    float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j0 < NP) {
      a = ld_x4(xrow + j0, nt);
      if (nd) d = ld4(drow + j0);
      if (na) an = ld_x4(arow + j0, nt);
    }
    xo[4 * q] = a.x; xo[4 * q + 1] = a.y; xo[4 * q + 2] = a.z; xo[4 * q + 3] = a.w;
    dout[4 * q] = d.x; dout[4 * q + 1] = d.y; dout[4 * q + 2] = d.z; dout[4 * q + 3] = d.w;
    ao[4 * q] = an.x; ao[4 * q + 1] = an.y; ao[4 * q + 2] = an.z; ao[4 * q + 3] = an.w;
  }
}

}  // namespace nep
