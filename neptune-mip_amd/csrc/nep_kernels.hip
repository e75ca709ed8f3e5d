// nep_kernels.hip — gfx950 kernels of one PDHG iteration on a batch of NEPTUNE LP relaxations.
//
// Iteration = one PDHG operator T (diagonally preconditioned; the primal set keeps every routing
// row on its simplex), wrapped in reflected restarted Halpern iterations (r2HPDHG):
//   x̂  = Π_simplex( x̄ − τ (cost_x − Kᵀ_x y) )           x_pass      (HBM-bound)
//   ẑ  = clip( z − τ γ² (cost_z − Kᵀ_z y) )              x_pass (c, moved) / node_pass (n) / scalar_pass
//   ŷ  = prox( y − σ ρ² K(2·[x̂,ẑ] − [x̄,z]) )             same split
//   w' = λ_k (2·T(w) − w) + (1 − λ_k) w_anchor,  λ_k = (k+1)/(k+2), k = iterations since restart
// ("plain" iterations take w' = T(w): the certificate iteration and the one before it, so the
// certificate's dual is a T output and satisfies the row sign constraints).
// K·[x̂, ẑ] is produced in the same passes that write the iterate (column sums, CPU sums, score
// row); the iterate's activity K w is kept in `kz` (the anchor's in `kza`, K is linear), so
// K(2ŵ − w) = 2·Kŵ − Kw costs no extra pass.  Built with NEP_INLINE_REFLECT, the per-(f, j) rows
// C1/C2/D1/D2 form K(2ŵ − w) in x_pass itself instead (column sums of m (2x̂ − x̄), old and new c /
// moved in registers) and skip their kz / kza.
//
// Launches per iteration: x_pass (one workgroup per (function f, LP slot): all routing rows of f,
// then the per-(f,j) variables c / moved_from / moved_to and rows C1/C2/D1/D2 of that f) and
// node_pass (per-node rows C3/C5/C6/C7 and n); scalar_pass on certificate iterations and on every
// step-2 iteration.  Every reduction has a fixed order: results are bitwise reproducible.
//
// Reference rows (core/solvers/neptune/utils): C1/C2 constraints_step1.py:5-15 (column sums),
// C3 :18-23, C4 :27-34 (the simplex), C5 :57-65 (CPU), C6/C7 :69-78; step 2 D1-D4
// constraints_step2.py:5-55, score rows :57-88.  Objectives objectives.py:4-63.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <algorithm>
#include <cmath>

#include "nep_internal.h"
#include "nep_device.h"

// NEP_INLINE_REFLECT (build flag, default off until the whole GPU suite has run on it):
// the C1/C2/D1/D2 duals take the reflected activity K(2ŵ - w) formed in x_pass instead of the tracked
// activities kz / kza (48 B per (f, j) and LP-iteration less)
#ifndef NEP_INLINE_REFLECT
#define NEP_INLINE_REFLECT 0
#endif
// NEP_XPASS_PREFETCH: the plain x_pass (rows of up to 512 destinations) loads each wave's NEXT routing row into
// registers while it works on the current one (5 waves per SIMD instead of 6).  1: the next row's x and delay row go
// out before the projection — measured slower (0.575 vs 0.545 ms per 29-slot launch, round 6; round 1 likewise).
// 2 (default since round 6): every load of the next row goes out after the projection and before the current row's
// stores, so no row waits for the previous row's stores to be acknowledged (the vector-memory counter counts stores,
// in order): 0.484 vs 0.512 ms per 32-slot launch on the whole-trace replay, the same iterations.
// 0: no prefetch (6 waves).
#ifndef NEP_XPASS_PREFETCH
#define NEP_XPASS_PREFETCH 2
#endif
// waves per SIMD the certificate x_pass is compiled for (build flag; 2: 210 VGPRs, no spills; 3: 168 VGPRs
// with 160 B/lane of spills, matching the 3 workgroups per CU its LDS allows)
#ifndef NEP_CHECK_WAVES
#define NEP_CHECK_WAVES 2
#endif
// waves per SIMD the plain x_pass (N <= 512) is compiled for (build flag for A/B)
#ifndef NEP_XPASS_WAVES
#define NEP_XPASS_WAVES 6
#endif
#ifndef NEP_XPASS_PF_WAVES   // (the same with a prefetch: its registers cost a wave)
#define NEP_XPASS_PF_WAVES 5
#endif
#ifndef NEP_XPASS_PF_ANCHOR  // (0, default: the late prefetch leaves a dense anchor row to the row's top — 90 instead
#define NEP_XPASS_PF_ANCHOR 0  //  of 96 VGPRs, 0.4955 vs 0.5044 ms per 32-slot launch; 1: prefetched with the rest)
#endif
#ifndef NEP_XPASS_PF_CPL1    // (the prefetch for rows of <= 256 destinations too: 256x128 product search, 20 s:
#define NEP_XPASS_PF_CPL1 1  //  9166 vs 8814 node LPs, the same incumbent and bound)
#endif

namespace nep {

// The certificate's pooled shift (one wave; x_pass, DESIGN.md §4 "Pooled shift"): S[j] the fp64
// column sums of f, pm[j] the pooled row's flow.  Deficits are served in j order, each from the
// donors in j order; deterministic.
// Deficits up to kShiftMax are served.  The shifted pooled row is written back into the stored iterate
// (x_pass, after the shift), so the shift may exceed fp32 rounding: pooled flow carries no cost, CPU load or
// score coefficient, and a donor keeps S >= c - eps, so every row the certificate checks holds as before.
constexpr double kShiftMax = 1e-3;
// the c a shift aims the column at: the iterate's c clamped into its node box and, on step 2, into the box
// the disruption rows imply with moved_from / moved_to fixed (constraints_step2.py:5-16: c <= old + ub_mf,
// c >= old - ub_mt — e.g. moved_to = 0 on an old placement forces c = 1)
__device__ __forceinline__ double c_target(const DeviceView &v, const double *zi, const double *lb, const double *ub,
                                           int f, int j) {
  const int k = v.il.oc + f * v.N + j;
  double lo = lb[k], hi = ub[k];
  if (v.step2) {
    const int idx = f * v.N + j;
    const double old = -v.lo[v.dl.oD1 + idx];
    lo = fmax(lo, old - ub[v.il.omt + idx]);
    hi = fmin(hi, old + ub[v.il.omf + idx]);
  }
  return fmin(fmax(zi[k], lo), hi);
}
__device__ __forceinline__ void pooled_shift(const DeviceView &v, int slot, int f, double *S, double *pm, int lane) {
  const int N = v.N;
  const double *zi = v.zi + slot * v.sint, *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  auto target = [&](int j) { return c_target(v, zi, lb, ub, f, j); };
  for (int j0 = 0; j0 < N; j0 += kWave) {
    const int j = j0 + lane;
    // deficits up to kShiftMax (the stored row takes the shift: see x_pass)
    const double need = j < N ? target(j) - v.eps - S[j] : 0.0;
    uint64_t mask = __ballot(need > 0.0 && need <= kShiftMax);
    while (mask) {
      const int k = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int jd = j0 + k;
      double want = target(jd) - v.eps - S[jd];   // (re-read: earlier transfers may have moved S[jd])
      for (int d0 = 0; d0 < N && want > 0.0; d0 += kWave) {
        const int d = d0 + lane;
        const double av = (d < N && d != jd) ? fmin(pm[d], S[d] + v.eps - target(d)) : 0.0;
        uint64_t dm = __ballot(av > 0.0);
        while (dm && want > 0.0) {
          const int kd = __builtin_ctzll(dm);
          dm &= dm - 1;
          const int dj = d0 + kd;
          const double t = fmin(want, __shfl(av, kd, kWave));
          if (lane == 0) {
            S[dj] -= t;
            pm[dj] -= t;
            S[jd] += t;
            pm[jd] += t;
          }
          want -= t;
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

// The certificate's loaded-row shift (one wave, after pooled_shift; DESIGN.md §4 "Pooled shift"): a deficit
// the pooled row could not serve — a function whose sources all carry workload, e.g. a placement forced
// open by moved_to = 0 on an old placement (payload.json's step 2) — is taken from the function's loaded
// rows at donor destinations with slack (S + eps above their own c), up to kShiftMax, written into the
// stored iterate (so the routing read back is the point the certificate checks).  Unlike pooled flow this
// moves CPU load (W[f, i] cpr per unit) and delay cost: the W-weighted column sums Wd and the objective /
// score partials take the exact fp32 changes of the two entries.  Deterministic (rows, donors in order).
__device__ __forceinline__ void loaded_shift(const DeviceView &v, int slot, int f, int r0, int nrows, float *x,
                                             double *S, double *Wd, double &dpobj, double &dscore, int lane) {
  const int N = v.N, NP = v.NP;
  const double *zi = v.zi + slot * v.sint, *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  auto target = [&](int j) { return c_target(v, zi, lb, ub, f, j); };
  for (int j0 = 0; j0 < N; j0 += kWave) {
    const int j = j0 + lane;
    const double need = j < N ? target(j) - v.eps - S[j] : 0.0;
    uint64_t mask = __ballot(need > 0.0 && need <= kShiftMax);
    while (mask) {
      const int k = __builtin_ctzll(mask);
      mask &= mask - 1;
      const int jd = j0 + k;
      double want = target(jd) - v.eps - S[jd];
      for (int rr = 0; rr < nrows && want > 0.0; ++rr) {
        const int r = r0 + rr;
        const RowInfo ri = v.rows[r];
        if (ri.src < 0) continue;
        float *xr = x + (int64_t)r * NP;
        const double m = ri.m;
        for (int d0 = 0; d0 < N && want > 0.0; d0 += kWave) {
          const int d = d0 + lane;
          const double av = (d < N && d != jd) ? fmin(m * (double)xr[d], S[d] + v.eps - target(d)) : 0.0;
          uint64_t dm = __ballot(av > 0.0);
          while (dm && want > 0.0) {
            const int kd = __builtin_ctzll(dm);
            dm &= dm - 1;
            const int dj = d0 + kd;
            const double t = fmin(want, __shfl(av, kd, kWave));
            if (lane == 0) {
              const float oj = xr[jd], od = xr[dj];
              const float nj = (float)((double)oj + t / m), nd = fmaxf((float)((double)od - t / m), 0.f);
              const double tj = (double)nj - oj, td = (double)od - nd;   // the exact fp32 changes
              xr[jd] = nj;
              xr[dj] = nd;
              S[jd] += m * tj;
              S[dj] -= m * td;
              Wd[jd] += (double)ri.w * tj;
              Wd[dj] -= (double)ri.w * td;
              const double dj_ = v.D[(int64_t)ri.src * NP + jd], dd_ = v.D[(int64_t)ri.src * NP + dj];
              dpobj += (double)ri.wobj * (dj_ * tj - dd_ * td);
              dscore += (double)ri.wsc * (dj_ * tj - dd_ * td);
            }
            want -= t;
          }
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// x_pass: one workgroup = all routing rows of ONE function f of one LP slot, then the
// per-(f, j) small variables of that f.
//  1. rows: each of the TW waves owns whole rows (N destinations = CPL float4 chunks per lane,
//     1 KiB per wave-instruction), projects each row on its simplex with Michelot's algorithm
//     (DPP sums + ballot counts), writes x̄' and accumulates the column sums (C1/C2) and
//     W-weighted sums (C5) into its own LDS row;
//  2. LDS reduction of the column sums across waves (fixed wave order);
//  3. per destination j: c[f,j] (+ moved_from/moved_to in step 2), the C1/C2 (D1/D2) duals,
//     the packed dual y1+y2 the next iteration's rows read, and f's share of the node rows
//     (memory, Σ_f c, CPU) for node_pass;
//  4. (init / certificate / step-2 iterations) the workgroup's scalar partials.
// ---------------------------------------------------------------------------------------------
// Occupancy: the plain iterations are held to <= 85 VGPRs (6 waves per SIMD; no spills at TW 4, 11
// VGPRs / 32 B per lane spilled at TW 8, which only runs for 2-3 slots where 6 waves keep 3
// workgroups per CU resident);
// measured at 512x256 / ~14 LPs per launch: 0.382 ms per launch vs 0.402 at the compiler's own 86
// VGPRs (5 waves) and 0.428 when forced to 8 waves (64 VGPRs + 68 B/lane of spills).  The
// certificate iterations (fp64 Lagrangian terms, 143 VGPRs) run at 3 waves per SIMD.  N > 512 (CPL 4, 8: 16 / 32
// destinations per lane) gets the register budget of 4 / 2 waves per SIMD: held to 6 waves those variants spilled
// 60 (CPL 4) to 280 (CPL 8) VGPRs per lane to scratch, and the 1024x512 lone root ran its TW 8 launches at 370 us
// (DESIGN.md §6 "N > 512").
// FIRST: the block's first iteration, the only one (with INIT) where a restart decided at the
// certificate iteration takes effect and the anchor is rewritten; the steady-state variant carries
// no restart code (fewer registers live).
template <int CPL, bool CHECK, bool INIT, bool FIRST, int TW>
__global__ __launch_bounds__(kWave * TW) __attribute__((amdgpu_waves_per_eu(
    CHECK ? NEP_CHECK_WAVES : (TW == 16 ? 4 : (CPL >= 8 ? 2 : (CPL >= 4 ? 4 : ((NEP_XPASS_PREFETCH && !FIRST && (CPL == 2 || (NEP_XPASS_PF_CPL1 && CPL == 1))) ? NEP_XPASS_PF_WAVES : NEP_XPASS_WAVES)))), 8)))
void x_pass(DeviceView v, const int32_t *__restrict__ slots, int plain, int it, int nslots, int nt_i) {
  const bool nt = nt_i != 0;
  constexpr int E = 4 * CPL;
  extern __shared__ __attribute__((aligned(16))) float lds[];   // [2][TW][NP] accumulators + [2][NP] constants
  __shared__ double lds_s[TW][NTS + NBS];
  // XCD-aware order (speed only; every (f, slot) pair is one workgroup either way): workgroup
  // ids are dealt round-robin over the 8 XCDs, so id -> p = (id % 8) * Q + id / 8 gives each XCD
  // a contiguous run of p = f * nslots + s, i.e. all the LP slots of the same functions back to
  // back on one XCD: the delay rows D[src, :] of a function's routing rows are then fetched into
  // that XCD's L2 once and re-read from it by the function's other slots.
  const int total = v.F * nslots, Q = (total + 7) / 8;
  const int p = (int)(blockIdx.x % 8) * Q + (int)(blockIdx.x / 8);
  if (p >= total) return;
  const int f = p / nslots;
  const int slot = slots[p - f * nslots];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int NP = v.NP, F = v.F, N = v.N;
  const float tau = INIT ? 0.f : (float)ctrl->tau;
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
  int32_t *__restrict__ acnt = v.acnt + (int64_t)slot * v.R;
  AnchorEnt *__restrict__ aent = v.aent + ((int64_t)slot * v.R) * kAnchorK;
  float *__restrict__ th_row = v.theta + (int64_t)slot * v.R;   // per-row simplex thresholds (hints)
  const uint8_t *__restrict__ mask = v.mask + slot * v.smask + (int64_t)f * NP;
  float *__restrict__ kty = v.kty + slot * v.skty;
  // polishing: objective off (cs = 0); at its first iteration the duals count as 0 (the originals are
  // kept in ybak), at the first iteration after it they are read back from ybak
  const int pol_sw = FIRST ? ctrl->polish_pending : 0;
  const bool pol_enter = pol_sw == 1, pol_leave = pol_sw == 2;
  const double *ybak = v.ybak + slot * v.sdual;
  const bool polishing = ctrl->polish != 0;
  const float cs = polishing ? 0.f : 1.f;
  // (oS, the step-2 score row, exists in step 2 only; step-2 LPs polish too: its dual is kept in ybak[oS]
  // by scalar_pass when polishing starts and read back here when it ends)
  const float ys = pol_enter ? 0.f
                             : ((pol_leave && v.step2) ? (float)ybak[v.dl.oS] : kty[(int64_t)F * NP + NP]);

  // Per-function column constants (packed duals kx = y1 + y2 and cy5 = cpr * y5) and the per-wave
  // column accumulators (C1/C2 column sums, C5 W-weighted sums) live in LDS, not in registers:
  // 32 fewer VGPRs per lane at CPL = 2, i.e. more waves per SIMD to keep HBM reads in flight.
  // Certificate iterations keep the column sums S[f, j] in fp64 (lSd, in place of lS): the
  // certificate's repaired point takes c from S exactly (pooled rows carry weights m ~ N, whose fp32
  // products would shift S by ~1e-5), and the constants in fp64 from the fp64 duals (lKd, lCd), so
  // the Lagrangian bound carries no fp32 rounding of y (|y1| can be large against the big-M rows).
  constexpr int SW = CHECK ? 2 : 1;   // words per column-sum accumulator (the CPU sums lW alike)
  float *lS = lds, *lW = lds + SW * TW * NP, *lK = lW + SW * TW * NP, *lC = lK + NP;
  double *lSd = reinterpret_cast<double *>(lS), *lWd = reinterpret_cast<double *>(lW);
  double *lKd = reinterpret_cast<double *>(lC + NP), *lCd = lKd + NP;
  double *lKr = lCd + NP;   // certificate: the repaired column prices s*[j] of f (DESIGN.md §4 "Dual repair")
  double *lPm = lKr + NP;   // certificate: the pooled row's flow m * x̂[pooled, j] (fp64; DESIGN.md §4 "Pooled shift")
  // The C1/C2 duals need the reflected activity K(2ŵ - w) only: the plain iterations accumulate the
  // reflected column sums m (2x̂ - x) in lS itself; the certificate ones, which keep the sums of x̂ in
  // fp64 for the repaired point, accumulate them beside it (lR, fp32 [TW][NP])
  float *lR = reinterpret_cast<float *>(lPm + NP);
  // the price of sum c the step-2 repair aims at (pre-update duals of D3a / D3b / D4)
  double lam_rep = 0.0;
  if (CHECK && v.step2 && !v.dred) {
    double lamk[kNLam];
    dblock_lambdas(v, v.y + slot * v.sdual, lamk);
    lam_rep = repair_lambda(lamk);
  }
  for (int j = threadIdx.x; j < NP; j += kWave * TW) {
    if (pol_leave) {
      const bool in = j < N;
      lK[j] = in ? (float)(ybak[v.dl.o1 + f * N + j] + ybak[v.dl.o2 + f * N + j]) : 0.f;
      lC[j] = in ? v.cpr[(int64_t)f * NP + j] * (float)ybak[v.dl.o5 + j] : 0.f;
    } else {
      lK[j] = pol_enter ? 0.f : kty[(int64_t)f * NP + j];
      lC[j] = pol_enter ? 0.f : v.cpr[(int64_t)f * NP + j] * kty[(int64_t)F * NP + j];
    }
    if (CHECK) {
      const double *yv = v.y + slot * v.sdual;
      const bool in = j < N;
      lKd[j] = in ? yv[v.dl.o1 + f * N + j] + yv[v.dl.o2 + f * N + j] : 0.0;
      lCd[j] = in ? (double)v.cpr[(int64_t)f * NP + j] * yv[v.dl.o5 + j] : 0.0;
      lKr[j] = in ? repaired_col_price(v, slot, f, j, lam_rep) : 0.0;
      lPm[j] = 0.0;
    }
  }
  const double ysd = (CHECK && v.step2) ? v.y[slot * v.sdual + v.dl.oS] : 0.0;
  uint32_t mbits = 0;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int j0 = 4 * (lane + kWave * q);
    if (j0 < NP) {
      const uchar4 m = *reinterpret_cast<const uchar4 *>(mask + j0);
      mbits |= (uint32_t)(m.x != 0) << (4 * q) | (uint32_t)(m.y != 0) << (4 * q + 1) |
               (uint32_t)(m.z != 0) << (4 * q + 2) | (uint32_t)(m.w != 0) << (4 * q + 3);
      if (CHECK) {
        double2 *pd = reinterpret_cast<double2 *>(lSd + wave * NP + j0);
        double2 *pe = reinterpret_cast<double2 *>(lWd + wave * NP + j0);
        pd[0] = pd[1] = pe[0] = pe[1] = make_double2(0.0, 0.0);
        if (NEP_INLINE_REFLECT) *reinterpret_cast<float4 *>(lR + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        *reinterpret_cast<float4 *>(lS + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4 *>(lW + wave * NP + j0) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  __syncthreads();
  // allowed destinations of f at this node: the same simplex support for every row of f
  int cnt_f = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) cnt_f += __popcll(__ballot((mbits >> e) & 1u));

  double s_score = 0.0, s_pobj = 0.0, s_lagr = 0.0, s_lagr_r = 0.0, s_lagr0 = 0.0, s_move = 0.0, s_dist = 0.0;
  const double s_empty = (cnt_f == 0 && threadIdx.x == 0) ? (double)nrows : 0.0;

  // (rows of up to 512 destinations: wider ones would spill)
  // (not the block's first iteration either: its restart code with the prefetch spills 41 VGPRs, 0.85 vs 0.57 ms)
  constexpr bool kPf = NEP_XPASS_PREFETCH && !CHECK && !FIRST && (CPL == 2 || (NEP_XPASS_PF_CPL1 && CPL == 1));
  // NEP_XPASS_PREFETCH == 2 ("late"): every load of the next row — its RowInfo, anchor count and pairs, threshold
  // hint, x, delay and dense anchor rows — goes out after this row's projection and BEFORE this row's stores, so the
  // wait for them at the next row's top need not wait for the stores (the vector-memory counter is in order and
  // counts stores): DESIGN.md §11 "x_pass store latency".  The arithmetic is the default's, value for value.
  constexpr bool kLate = NEP_XPASS_PREFETCH == 2 && kPf;
  float pfx[E], pfd[E], pfa[E];   // (unused without NEP_XPASS_PREFETCH: removed by the compiler)
  RowInfo pri{};
  int pacn = 0;
  float pth = 0.f;
  AnchorEnt pae{0, 0.f};
  auto row_nd = [&](const RowInfo &q) { return q.src >= 0 && (q.wobj != 0.f || q.wsc != 0.f); };
  auto prefetch = [&](int rn) {
    const RowInfo q = v.rows[rn];
    int qa = 0;
    if (need_anchor) qa = NEP_SPARSE_ANCHOR ? __builtin_amdgcn_readfirstlane(acnt[rn]) : kAnchorDense;
    load_row<CPL>(x + (int64_t)rn * NP, v.D + (int64_t)(q.src < 0 ? 0 : q.src) * NP, xa + (int64_t)rn * NP, row_nd(q),
                  NEP_XPASS_PF_ANCHOR && need_anchor && qa > kAnchorK, nt, lane, NP, pfx, pfd, pfa);
    AnchorEnt qe{0, 0.f};
    if (need_anchor && qa <= kAnchorK && lane < qa) qe = aent[(int64_t)rn * kAnchorK + lane];
    pth = th_row[rn];
    pri = q;
    pacn = qa;
    pae = qe;
  };
  if (kLate && wave < nrows) {
    prefetch(r0 + wave);
  } else if (kPf && wave < nrows) {
    const RowInfo q = v.rows[r0 + wave];
    float dummy[E];
    load_row<CPL>(x + (int64_t)(r0 + wave) * NP, v.D + (int64_t)(q.src < 0 ? 0 : q.src) * NP, xa, row_nd(q), false, nt,
                  lane, NP, pfx, pfd, dummy);
  }
  for (int rr = wave; rr < nrows; rr += TW) {
    const int r = r0 + rr;
    const RowInfo ri = kLate ? pri : v.rows[r];
    const bool nd = row_nd(ri);
    float xc[E], dc[E], ac[E];
    // anchor row: kept sparse (<= kAnchorK (j, value) pairs, lanes 0..cnt-1 load one each) or dense
    int acn = 0;
    if (kLate) acn = pacn;
    else if (need_anchor) acn = NEP_SPARSE_ANCHOR ? __builtin_amdgcn_readfirstlane(acnt[r]) : kAnchorDense;
    if (kLate) {
#pragma unroll
      for (int e = 0; e < E; ++e) { xc[e] = pfx[e]; dc[e] = pfd[e]; ac[e] = NEP_XPASS_PF_ANCHOR ? pfa[e] : 0.f; }
      if (!NEP_XPASS_PF_ANCHOR && need_anchor && acn > kAnchorK) {   // (A/B: the dense anchor loaded here instead)
        float d0[E], d1[E];
        load_row<CPL>(xa + (int64_t)r * NP, v.D, xa + (int64_t)r * NP, false, false, nt, lane, NP, ac, d0, d1);
      }
    } else if (kPf) {
      // this row came in with the previous one; the next row's loads go out now, ahead of the projection
#pragma unroll
      for (int e = 0; e < E; ++e) { xc[e] = pfx[e]; dc[e] = pfd[e]; ac[e] = 0.f; }
      if (need_anchor && acn > kAnchorK) {
        float d0[E], d1[E];
        load_row<CPL>(xa + (int64_t)r * NP, v.D, xa + (int64_t)r * NP, false, false, nt, lane, NP, ac, d0, d1);
      }
      if (rr + TW < nrows) {
        const RowInfo q = v.rows[r + TW];
        float dummy[E];
        load_row<CPL>(x + (int64_t)(r + TW) * NP, v.D + (int64_t)(q.src < 0 ? 0 : q.src) * NP, xa, row_nd(q), false,
                      nt, lane, NP, pfx, pfd, dummy);
      }
    } else {
      // (default: no software prefetch of the next row — the registers it costs are worth more as occupancy,
      // 0.575 vs 0.591 ms per launch in round 1; other waves hide the latency)
      load_row<CPL>(x + (int64_t)r * NP, v.D + (int64_t)(ri.src < 0 ? 0 : ri.src) * NP, xa + (int64_t)r * NP, nd,
                    need_anchor && acn > kAnchorK, nt, lane, NP, xc, dc, ac);
    }
    if (need_anchor && acn <= kAnchorK) {
      AnchorEnt ae{0, 0.f};
      if (kLate) ae = pae;
      else if (lane < acn) ae = aent[(int64_t)r * kAnchorK + lane];
      // scatter the pairs into the lanes that own their destinations (ac is zero from load_row)
      // (destination j lives in lane (j >> 2) & 63, register 4 * (j >> 8) + (j & 3): see load_row)
      for (int k = 0; k < acn; ++k) {
        const int jk = __builtin_amdgcn_readlane(ae.j, k);
        const float vk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ae.v), k));
        const int ek = ((jk >> 8) << 2) | (jk & 3);   // wave-uniform
        const bool mine = lane == ((jk >> 2) & (kWave - 1));
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (e == ek) ac[e] = mine ? vk : ac[e];
      }
    }
    const float m = ri.m, w = ri.w, wobj = ri.wobj, wsc = ri.wsc;
    const float wg = polishing ? 0.f : wobj;   // objective off while polishing (a select on the uniform row value)
    float kx[E], cy5[E];
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), c = a;
      if (j0 < NP) {
        a = *reinterpret_cast<const float4 *>(lK + j0);
        c = *reinterpret_cast<const float4 *>(lC + j0);
      }
      kx[4 * q] = a.x; kx[4 * q + 1] = a.y; kx[4 * q + 2] = a.z; kx[4 * q + 3] = a.w;
      cy5[4 * q] = c.x; cy5[4 * q + 1] = c.y; cy5[4 * q + 2] = c.z; cy5[4 * q + 3] = c.w;
    }
    // gradient step (reduced cost of x̄[r, j] = cost − Kᵀy)
    float vv[E];
    float s = 0.f;
    const float gs = wsc * ys;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float g = wg * dc[e] - (m * kx[e] + w * cy5[e] + gs * dc[e]);
      vv[e] = xc[e] - tau * g;
      if ((mbits >> e) & 1u) s += vv[e];
    }
    if (CHECK) {
      // Lagrangian term of this row: min over the simplex of the reduced cost, in fp64, at the PDHG
      // duals and at the repaired column prices
      double gmin = INFINITY, gmin_r = INFINITY, gmin0 = INFINITY;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if ((mbits >> e) & 1u) {
          const int j = 4 * (lane + kWave * (e / 4)) + (e & 3);
          const double g0 = (double)wobj * dc[e] - ((double)w * lCd[j] + (double)wsc * ysd * dc[e]);
          gmin = fmin(gmin, g0 - (double)m * lKd[j]);
          gmin_r = fmin(gmin_r, g0 - (double)m * lKr[j]);
          gmin0 = fmin(gmin0, g0 - (double)wobj * dc[e] - (double)m * lKd[j]);   // objective off
        }
      }
      gmin = wave_min_d(gmin);
      gmin_r = wave_min_d(gmin_r);
      gmin0 = wave_min_d(gmin0);
      if (lane == 0) { s_lagr += gmin; s_lagr_r += gmin_r; s_lagr0 += gmin0; }
    }
    // Projection onto {x >= 0, sum x = 1} over the allowed destinations: the threshold theta is
    // the root of f(t) = sum_j max(v_j - t, 0) - 1 (convex, decreasing).  Michelot's iteration is
    // Newton's method on f from the left (t <- (S(t) - 1) / c(t), S/c = sum/count of v > t) and is
    // exact once the count stops changing, but it can take O(N) steps when many values sit just
    // above the root.  Safeguard: after 4 Newton steps, alternate bisection steps on the bracket
    // [lo, hi] (f(lo) >= 0 > f(hi), width <= 1 from [vmax - 1, vmax]) with Newton steps.  Every step
    // costs one DPP sum and E ballots; the converged theta is the same (S* - 1) / |S*| Michelot
    // returns, summed in the same order.
    float theta = INFINITY;
    if (cnt_f > 0) {
      float vm = -INFINITY;
#pragma unroll
      for (int e = 0; e < E; ++e)
        if ((mbits >> e) & 1u) vm = fmaxf(vm, vv[e]);
      // Start from this row's threshold of the previous iteration when it is usable: one pass gives
      // S and c at theta_prev, the first Newton step from there is the tangent root (left of the
      // root from either side, f being convex), and the support usually stops changing one pass
      // later.  Cold rows start from -inf (S = sum of all allowed values, c = cnt_f).  Either way
      // the loop ends on the same exact (S* - 1) / |S*|, so the start only changes the pass count.
      const float th0 = kLate ? pth : th_row[r];
      float lo_s = 0.f;
      int lo_c = 0;
      if (!INIT && th0 > -INFINITY && th0 < INFINITY) {   // false for NaN (no hint yet)
        float s0 = 0.f;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool in = ((mbits >> e) & 1u) && vv[e] > th0;
          if (in) s0 += vv[e];
          lo_c += __popcll(__ballot(in));
        }
        lo_s = wave_sum_u(s0);
      }
      if (lo_c == 0) {                              // no hint, or every value at or below it
        lo_s = wave_sum_u(s);
        lo_c = cnt_f;
      }
      float hi = INFINITY;                          // right bracket max(v): reduced only if bisection is needed
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
          if (c2 == lo_c || c2 == 0) break;   // support unchanged: t is the exact threshold
          lo = t; lo_s = s2; lo_c = c2;
        } else if (s2 - t * (float)c2 - 1.f >= 0.f && c2 > 0) {
          lo = t; lo_s = s2; lo_c = c2;
        } else {
          hi = t;
        }
      }
    }
    if (kLate && rr + TW < nrows) prefetch(r + TW);   // (before this row's first store)
    if (lane == 0) th_row[r] = theta;
    float xn[E];
    if (CHECK && cnt_f > 0) {
      // certificate iterations: the threshold again in fp64 over the support the fp32 search found, so the
      // stored row — the certificate's point — sums to 1 within the fp32 rounding of its entries (C4,
      // constraints_step1.py:27-34).  An fp32 threshold over ~N active entries leaves |sum - 1| ~ N ulps: 1.2e-5
      // on the pooled rows of the Alibaba-shape 1024x512 models (W == 0: one row of 1024 entries per function)
      // Michelot passes in fp64 from the fp32 support until the support {v > th} is stable (round-5 ADVICE:
      // applying th64 to every masked entry moved entries across the fp32 support's edge); the final threshold
      // is always the one computed from the final support, whose entries outside stay 0
      double th64 = (double)theta;
      uint32_t sup = 0xffffffffu;
#pragma unroll 1
      for (int it = 0; it < 4; ++it) {
        double s64 = 0.0;
        int c64 = 0;
        uint32_t ns = 0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const bool in = ((mbits >> e) & 1u) && (double)vv[e] > th64;
          if (in) {
            s64 += (double)vv[e];
            ns |= 1u << e;
          }
          c64 += __popcll(__ballot(in));
        }
        if (__ballot(ns != sup) == 0) break;
        sup = ns;
        s64 = wave_sum_d(s64);
        if (c64 > 0) th64 = (s64 - 1.0) / (double)c64;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) xn[e] = ((sup >> e) & 1u) ? fmaxf((float)((double)vv[e] - th64), 0.f) : 0.f;
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) xn[e] = ((mbits >> e) & 1u) ? fmaxf(vv[e] - theta, 0.f) : 0.f;
    }
    if (CHECK && ri.src < 0) {   // the pooled row of f: its flow, for the certificate's pooled shift
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = 4 * (lane + kWave * (e / 4)) + (e & 3);
        if (j < NP) lPm[j] = (double)m * (double)xn[e];
      }
    }

    // anchor row: needed by the Halpern combination and by the certificate's restart distance
    float xav[E];
#pragma unroll
    for (int e = 0; e < E; ++e) xav[e] = need_anchor ? ac[e] : (INIT ? xn[e] : xc[e]);
    if (CHECK && !restart) {
      double dd = 0.0;
#pragma unroll
      for (int e = 0; e < E; ++e) { const double t = (double)xn[e] - xav[e]; dd += t * t; }
      s_dist += dd;
    }
    float *xrow = x + (int64_t)r * NP;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      if (j0 < NP) {
        float o[4], rf[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int e = 4 * q + t;
          rf[t] = 2.f * xn[e] - xc[e];   // reflected point 2x̂ - x
          o[t] = halp ? lam * rf[t] + (1.f - lam) * xav[e] : xn[e];
        }
        st_x4(xrow + j0, f32x4{o[0], o[1], o[2], o[3]}, nt);
        // column sums m x̂, or the reflected m (2x̂ - x) (plain iterations: lS; certificate iterations: lR)
        if (NEP_INLINE_REFLECT) {
          float4 *pr = reinterpret_cast<float4 *>((CHECK ? lR : lS) + wave * NP + j0);
          float4 c = *pr;
          c.x += m * rf[0]; c.y += m * rf[1]; c.z += m * rf[2]; c.w += m * rf[3];
          *pr = c;
        }
      }
    }
    if (restart) {
      // new anchor = xav: compacted to (j, value) pairs when it has <= kAnchorK nonzeros (a point on
      // the simplex usually has a handful), else written dense.  Same values either way.
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
    float sc = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int j0 = 4 * (lane + kWave * q);
      if (j0 < NP) {
        const float *xq = xn + 4 * q;
        if (CHECK) {
          double2 *pd = reinterpret_cast<double2 *>(lSd + wave * NP + j0);
          double2 *pe = reinterpret_cast<double2 *>(lWd + wave * NP + j0);
          double2 a0 = pd[0], a1 = pd[1], b0 = pe[0], b1 = pe[1];
          const double md = m, wd = w;
          a0.x += md * xq[0]; a0.y += md * xq[1]; a1.x += md * xq[2]; a1.y += md * xq[3];
          b0.x += wd * xq[0]; b0.y += wd * xq[1]; b1.x += wd * xq[2]; b1.y += wd * xq[3];
          pd[0] = a0; pd[1] = a1; pe[0] = b0; pe[1] = b1;
        } else if (NEP_INLINE_REFLECT) {
          float4 *pw = reinterpret_cast<float4 *>(lW + wave * NP + j0);
          float4 b = *pw;
          b.x += w * xq[0]; b.y += w * xq[1]; b.z += w * xq[2]; b.w += w * xq[3];
          *pw = b;
        } else {
          float4 *ps = reinterpret_cast<float4 *>(lS + wave * NP + j0);
          float4 *pw = reinterpret_cast<float4 *>(lW + wave * NP + j0);
          float4 a = *ps, b = *pw;
          a.x += m * xq[0]; a.y += m * xq[1]; a.z += m * xq[2]; a.w += m * xq[3];
          b.x += w * xq[0]; b.y += w * xq[1]; b.z += w * xq[2]; b.w += w * xq[3];
          *ps = a;
          *pw = b;
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) sc += dc[e] * xn[e];
    s_score += (double)wsc * (double)sc;
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

  // cross-wave reduction of the column partials (each wave's accumulators are in LDS)
  __syncthreads();
  if (CHECK) {
    // certificate: the column / CPU sums of f in fp64, reduced over the waves into wave 0's slots, then
    // the pooled shift (DESIGN.md §4 "Pooled shift"): a destination j whose c the certificate wants
    // at ~1 (the iterate's c) but whose fp32 column sum S_j fell short of c - eps by rounding takes the
    // missing flow from the pooled row (zero-workload sources: no cost, CPU or score coefficient) at a
    // destination with slack (S + eps above its own c); the certificate point is x̂ with the pooled row
    // shifted by those fp64 amounts, the same simplex and the same objective.  Without it a deficit of
    // d costs (2 F N - 1) d on step 2 (moved_to + allocated), ~1e-4 at 64x32 from fp32 rounding alone.
    for (int j = threadIdx.x; j < N; j += kWave * TW) {
      double Sd = 0.0, Ud = 0.0;
#pragma unroll
      for (int wv = 0; wv < TW; ++wv) {
        Sd += lSd[wv * NP + j];
        Ud += lWd[wv * NP + j];
      }
      lSd[j] = Sd;
      lWd[j] = Ud;
    }
    __syncthreads();
    if (wave == 0) {
      pooled_shift(v, slot, f, lSd, lPm, lane);
      // (the pooled row's own write-back below rewrites only its row; the loaded rows are written in place)
      double dpo = 0.0, dsc = 0.0;
      loaded_shift(v, slot, f, r0, nrows, x, lSd, lWd, dpo, dsc, lane);
      if (lane == 0) {
        s_pobj += dpo;
        s_score += dsc;
      }
      // the certificate's point is the STORED iterate (this plain iteration's x̂): the pooled row takes
      // the shifted flows, so the routing a caller reads back (nep_lp_get_rows / routing entries) is
      // the point the certificate checked, not one kShiftMax short of it on a column.  Unshifted
      // entries rewrite the same value: (float)((m * x̂) / m) == x̂ exactly (the product is exact in fp64).
      const int rp = r0 + nrows - 1;
      if (nrows > 0 && v.rows[rp].src < 0) {
        const double mp = v.rows[rp].m;
        for (int j = lane; j < N; j += kWave) x[(int64_t)rp * NP + j] = (float)(lPm[j] / mp);
      }
    }
    __syncthreads();
  }

  // per-(f, j) small variables and rows
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  const double taud = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool copy_anchor = restart;
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  double *np_ = v.npart + slot * v.snpart + (int64_t)f * 2 * NP;
  const double memf = v.mem_f[f];
  // (step-2 scalar rows, owned by scalar_pass: 0 at the first polishing iteration, kept values after it)
  const double *yst = pol_leave ? ybak : y;
  const double yD3a = (v.step2 && !pol_enter) ? yst[dl.oD3a] : 0.0, yD3b = (v.step2 && !pol_enter) ? yst[dl.oD3b] : 0.0;
  const double yD4 = (v.step2 && !pol_enter) ? yst[dl.oD4] : 0.0;
  const double csd = cs;   // polishing: small-variable costs off as well
  SmallAcc a;
  double sumc = 0.0, sumc_rep = 0.0;
  // step-2 certificate: the disruption block's exact terms per candidate price (PDHG / repaired duals)
  // and f's share of the node box of sum c
  double lamk[kNLam], dlk[kNLam], dlkr[kNLam], dtlo = 0.0, dthi = 0.0;
#pragma unroll
  for (int q = 0; q < kNLam; ++q) { lamk[q] = 0.0; dlk[q] = dlkr[q] = 0.0; }
  if (CHECK && v.step2 && !v.dred) dblock_lambdas(v, y, lamk);
  for (int j = threadIdx.x; j < N; j += kWave * TW) {
    float Sf = 0.f, Uf = 0.f;   // (plain iterations: Sf is the reflected column sum)
    double Sd = 0.0, Ud = 0.0;
    if (CHECK) {
      Sd = lSd[j];   // reduced (and pooled-shifted) above
      Ud = lWd[j];
#pragma unroll
      for (int wv = 0; wv < TW && NEP_INLINE_REFLECT; ++wv) Sf += lR[wv * NP + j];
    } else {
#pragma unroll
      for (int wv = 0; wv < TW; ++wv) {
        Sf += lS[wv * NP + j];
        Uf += lW[wv * NP + j];
      }
    }
    const double S = CHECK ? Sd : (double)Sf;   // column sum of x̂ (tracked-activity build)
    const double Sr = (double)Sf;               // reflected column sum of m (2x̂ - x) (NEP_INLINE_REFLECT)
    const double U = CHECK ? Ud * (double)v.cpr[(int64_t)f * NP + j] : (double)(Uf * v.cpr[(int64_t)f * NP + j]);
    const int idx = f * N + j;
    // (polishing: at its first iteration every dual counts as 0 — this f's rows C1/C2 are kept in
    // ybak, node_pass keeps the node rows — and after it they are read back)
    const double *ysrc = pol_leave ? ybak : y;
    double y1 = ysrc[dl.o1 + idx], y2 = ysrc[dl.o2 + idx];
    double y3 = ysrc[dl.o3 + j];
    double y6 = v.has_n ? ysrc[dl.o6 + j] : 0.0;
    double y7 = v.has_n ? ysrc[dl.o7 + j] : 0.0;
    if (pol_enter) {
      v.ybak[slot * v.sdual + dl.o1 + idx] = y1;
      v.ybak[slot * v.sdual + dl.o2 + idx] = y2;
      y1 = y2 = y3 = y6 = y7 = 0.0;
    }
    double kty_c = -v.M * y1 - y2 + memf * y3 + y6 + y7;
    // reduced step-2 block: c's own cost (which the objective-off Lagrangian takes out of rc as well), and the
    // row sum c's dual (D4's slot) in its reduced cost
    double dcost = 0.0, dconst = 0.0;
    if (__builtin_expect(v.dred, 0)) {
      dcost = dred_cost(v, lb, idx, dconst);
      kty_c += yD4;
    }
    if (CHECK && v.dred) {
      // the bound's small-variable terms at the repaired duals, as on step 1 with c's own cost and constant
      const double sr = lKr[j];
      const double rcr = price_rc(repaired_c_base(v, slot, f, j) + csd * dcost - yD4, sr, v.M);
      a.lagrR += fmin(lb[il.oc + idx] * rcr, ub[il.oc + idx] * rcr) - v.eps * fmax(sr, 0.0) + csd * dconst;
      a.lagr += csd * dconst;
    } else if (CHECK) {
      // the bound's small-variable terms at the repaired duals (DESIGN.md §4 "Dual repair"), and on
      // step 2 the disruption block kept exact (dblock_item) at both the PDHG and the repaired duals
      const double sr = lKr[j];
      const double rcr = price_rc(repaired_c_base(v, slot, f, j), sr, v.M);
      const double clb = lb[il.oc + idx], cub = ub[il.oc + idx];
      a.lagrR -= v.eps * fmax(sr, 0.0);
      if (!v.step2) {
        a.lagrR += fmin(clb * rcr, cub * rcr);
      } else {
        const double r0 = v.cost_int[il.oc + idx] - kty_c;   // c's reduced cost without the D rows
        const double old = -v.lo[dl.oD1 + idx];
        const double lmf = lb[il.omf + idx], lmt = lb[il.omt + idx];
        const double clo = fmax(clb, old - ub[il.omt + idx]), chi = fmin(cub, old + ub[il.omf + idx]);
        const double cmf = v.cost_int[il.omf + idx], cmt = v.cost_int[il.omt + idx];
        dtlo += clb;
        dthi += cub;
#pragma unroll
        for (int q = 0; q < kNLam; ++q) {
          dlk[q] += dblock_item(r0, lamk[q], old, cmf, lmf, cmt, lmt, clo, chi);
          dlkr[q] += dblock_item(rcr, lamk[q], old, cmf, lmf, cmt, lmt, clo, chi);
        }
      }
    }
    double yd1 = 0.0, yd2 = 0.0;
    if (v.step2 && !v.dred) {
      yd1 = ysrc[dl.oD1 + idx];
      yd2 = ysrc[dl.oD2 + idx];
      if (pol_enter) {   // D1/D2 rows of this f: kept, the feasibility problem's from 0
        v.ybak[slot * v.sdual + dl.oD1 + idx] = yd1;
        v.ybak[slot * v.sdual + dl.oD2 + idx] = yd2;
        yd1 = yd2 = 0.0;
      }
      kty_c += -yd1 + yd2 - yD3a + yD3b + v.sigma4 * yD4;
    }
    const double c_old = NEP_INLINE_REFLECT ? zi[il.oc + idx] : 0.0;
    ZPre pc = primal_pre(v, zi, zia, lb, ub, il.oc + idx, copy_anchor);
    if (v.dred) pc.cost = dcost;
    const double cn = primal_step_p<CHECK>(zi, zia, il.oc + idx, csd * pc.cost - kty_c, pc, taud, copy_anchor, halp,
                                           lamd, a, v.step2 && !v.dred);
    const double c2 = 2.0 * cn - c_old;   // reflected c
    double y1n, y2n;
    if (NEP_INLINE_REFLECT) {
      y1n = dual_step_refl<CHECK, INIT>(v, y, ya, dl.o1 + idx, Sr - v.M * c2, y1, sigma, copy_anchor, halp, lamd, a);
      y2n = dual_step_refl<CHECK, INIT>(v, y, ya, dl.o2 + idx, Sr - c2, y2, sigma, copy_anchor, halp, lamd, a);
    } else {
      y1n = dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o1 + idx, S - v.M * cn, y1, sigma, copy_anchor, halp, lamd, a);
      y2n = dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.o2 + idx, S - cn, y2, sigma, copy_anchor, halp, lamd, a);
    }
    if (v.dred) {
      // (moved_from / moved_to are not iterated: their LP optimum follows from c, the certificate below)
    } else if (v.step2 && !NEP_INLINE_REFLECT) {
      const double mfn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omf + idx, csd * v.cost_int[il.omf + idx] - yd1, taud,
                                            copy_anchor, halp, lamd, a, true);
      const double mtn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omt + idx, csd * v.cost_int[il.omt + idx] - yd2, taud,
                                            copy_anchor, halp, lamd, a, true);
      dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD1 + idx, mfn - cn, yd1, sigma, copy_anchor, halp, lamd, a, true);
      dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD2 + idx, mtn + cn, yd2, sigma, copy_anchor, halp, lamd, a, true);
    } else if (v.step2) {
      const double mf_old = zi[il.omf + idx], mt_old = zi[il.omt + idx];
      const double mfn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omf + idx, csd * v.cost_int[il.omf + idx] - yd1, taud,
                                            copy_anchor, halp, lamd, a, true);
      const double mtn = primal_step<CHECK>(v, zi, zia, lb, ub, il.omt + idx, csd * v.cost_int[il.omt + idx] - yd2, taud,
                                            copy_anchor, halp, lamd, a, true);
      dual_step_refl<CHECK, INIT>(v, y, ya, dl.oD1 + idx, (2.0 * mfn - mf_old) - c2, yd1, sigma, copy_anchor, halp,
                                  lamd, a, true);
      dual_step_refl<CHECK, INIT>(v, y, ya, dl.oD2 + idx, (2.0 * mtn - mt_old) + c2, yd2, sigma, copy_anchor, halp,
                                  lamd, a, true);
    }
    kty[(int64_t)f * NP + j] = (float)(y1n + y2n);
    np_[j] = cn;                 // node_pass forms the memory share mem_f * c itself
    np_[NP + j] = U;
    sumc += cn;
    if (CHECK) {
      // Certificate point: the routing x̂ of this iteration with the small variables REPAIRED, in
      // dependency order, onto the rows each one closes: c = the T output clamped into
      // [S/M, S + eps] (C1/C2) within the node box, then the cheapest mf = max(lb, c - old),
      // mt = max(lb, old - c) (D1/D2; both cost F*N).  At convergence the clamp moves c by the PDHG
      // residual only, so the repaired point keeps the iterate's (near-optimal) choices; an empty
      // interval is a violation of the x-driven row.
      double loc = fmax(lb[il.oc + idx], S / v.M), hic = fmin(ub[il.oc + idx], S + v.eps);
      if (v.step2) {   // within the box the D rows imply at the node's moved_from / moved_to bounds, if any
        const double old = -v.lo[dl.oD1 + idx];
        const double dlo = old - ub[il.omt + idx], dhi = old + ub[il.omf + idx];
        if (fmax(loc, dlo) <= fmin(hic, dhi)) {
          loc = fmax(loc, dlo);
          hic = fmin(hic, dhi);
        }
      }
      const double cr = loc > hic ? loc : fmin(fmax(cn, loc), hic);
      if (v.step2) {
        const double old = -v.lo[dl.oD1 + idx];
        const double mfr = fmax(lb[il.omf + idx], cr - old), mtr = fmax(lb[il.omt + idx], old - cr);
        v.zr[slot * v.sint + il.omf + idx] = mfr;
        v.zr[slot * v.sint + il.omt + idx] = mtr;
        if (v.dred) {   // (not iterated: the iterate carries the last certificate's values)
          zi[il.omf + idx] = mfr;
          zi[il.omt + idx] = mtr;
        }
        a.res = fmax(a.res, fmax(mfr - ub[il.omf + idx], mtr - ub[il.omt + idx]));
        a.pobj += v.cost_int[il.omf + idx] * mfr + v.cost_int[il.omt + idx] * mtr;
      }
      a.res = fmax(a.res, loc - hic);   // absolute: a fixed-open (f, j) needs flow >= c - eps
      a.pobj += v.cost_int[il.oc + idx] * cr;
      v.zr[slot * v.sint + il.oc + idx] = cr;
      sumc_rep += cr;
      double *rp = v.rpart + slot * v.srpart + (int64_t)f * 2 * NP;
      rp[j] = memf * cr;
      rp[NP + j] = cr;
    }
  }

  // scalar partials of this (f, slot): read by scalar_pass on init / certificate / step-2 iterations
  if (!(INIT || CHECK || v.step2)) return;
  double vals[NTS + NBS];
  vals[TS_SCORE] = s_score;
  vals[TS_POBJ] = s_pobj;
  vals[TS_LAGR] = s_lagr;
  vals[TS_MOVE] = s_move;
  vals[TS_DIST] = s_dist;
  vals[TS_EMPTY] = s_empty;
  vals[NTS + BS_SUMC_NEW] = sumc;
  vals[NTS + BS_SCORE_N] = 0.0;
  vals[NTS + BS_LAGR] = a.lagr;
  vals[NTS + BS_POBJ] = a.pobj;
  vals[NTS + BS_RES] = a.res;
  vals[NTS + BS_MOVE_Z] = a.mvz;
  vals[NTS + BS_MOVE_Y] = a.mvy;
  vals[NTS + BS_DIST_Z] = a.dsz;
  vals[NTS + BS_DIST_Y] = a.dsy;
  vals[NTS + BS_SUMC_REP] = sumc_rep;
  vals[NTS + BS_SCORE_N_REP] = 0.0;
  vals[NTS + BS_LAGR_D] = a.lagrD;
  vals[TS_LAGR_REP] = s_lagr_r;
  vals[NTS + BS_LAGR_REP] = a.lagrR;
  vals[TS_LAGR0] = s_lagr0;
  vals[NTS + BS_LAGR0] = a.lagr0;
  vals[NTS + BS_TLO] = dtlo;
  vals[NTS + BS_THI] = dthi;
#pragma unroll
  for (int q = 0; q < kNLam; ++q) {
    vals[NTS + BS_LK0 + q] = dlk[q];
    vals[NTS + BS_LKR0 + q] = dlkr[q];
  }
  constexpr int NW = NTS + NBS;
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    const bool needed = INIT || CHECK || k == TS_SCORE || k == NTS + BS_SUMC_NEW;
    double t = 0.0;
    if (needed) t = (k == NTS + BS_RES) ? wave_max_d(vals[k]) : wave_sum_d(vals[k]);
    if (lane == 0) lds_s[wave][k] = t;
  }
  __syncthreads();
  const int k = threadIdx.x;
  if (k < NW) {
    double t = 0.0;
#pragma unroll
    for (int wv = 0; wv < TW; ++wv) t = (k == NTS + BS_RES) ? fmax(t, lds_s[wv][k]) : t + lds_s[wv][k];
    if (k < NTS) v.tpart[slot * v.stpart + (int64_t)f * NTS + k] = t;
    else v.bpart[slot * v.sbpart + (int64_t)f * NBS + (k - NTS)] = t;
  }
}

template <bool ALL>
__device__ __forceinline__ void write_bpart(double *bp, const SmallAcc &a, double sumc, double score_n,
                                            double score_n_rep, int lane) {
  double vals[NBS];
  vals[BS_SUMC_REP] = 0.0;
  vals[BS_SCORE_N_REP] = score_n_rep;
  vals[BS_SUMC_NEW] = sumc;
  vals[BS_SCORE_N] = score_n;
  vals[BS_LAGR] = a.lagr;
  vals[BS_POBJ] = a.pobj;
  vals[BS_RES] = a.res;
  vals[BS_MOVE_Z] = a.mvz;
  vals[BS_MOVE_Y] = a.mvy;
  vals[BS_DIST_Z] = a.dsz;
  vals[BS_DIST_Y] = a.dsy;
  vals[BS_LAGR_D] = a.lagrD;
  vals[BS_LAGR_REP] = a.lagrR;
  vals[BS_LAGR0] = a.lagr0;
  vals[BS_TLO] = vals[BS_THI] = 0.0;
#pragma unroll
  for (int q = 0; q < kNLam; ++q) vals[BS_LK0 + q] = vals[BS_LKR0 + q] = 0.0;
  // plain step-2 iterations: scalar_pass reads only the row fields (ALL = false)
#pragma unroll
  for (int k = 0; k < NBS; ++k) {
    if (!ALL && k != BS_SCORE_N && k != BS_SUMC_NEW) continue;
    const double t = (k == BS_RES) ? wave_max_d(vals[k]) : wave_sum_d(vals[k]);
    if (lane == 0) bp[k] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// node_pass: one workgroup per (slot, block of 64 nodes j): the waves sum the per-function
// shares of the node rows (fixed order), then wave 0 updates rows C3 (memory), C5 (CPU), n and
// C6/C7.
// ---------------------------------------------------------------------------------------------
template <bool CHECK, bool INIT>
__global__ __launch_bounds__(kNodeThreads) void node_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                          int plain, int it) {
  // kNodeJ nodes per workgroup (so a lone LP still spreads its F x 3 x N shares over N / kNodeJ
  // workgroups): thread t sums the shares of node t % kNodeJ over function group t / kNodeJ
  constexpr int NG = kNodeThreads / kNodeJ;
  __shared__ double red[5][NG][kNodeJ];
  const int jb = blockIdx.x;
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  const int NP = v.NP, F = v.F;
  const DualLayout &dl = v.dl;
  const IntLayout &il = v.il;
  const bool copy_anchor = INIT || (first && ctrl->restart_pending);
  double *zi = v.zi + slot * v.sint, *zia = v.zia + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  double *y = v.y + slot * v.sdual, *ya = v.ya + slot * v.sdual, *kz = v.kz + slot * v.sdual;
  double *kza = v.kza + slot * v.sdual;
  // wave 0, lane (< kNodeJ) = node: issue every load of the node's rows now, ahead of the partial sums
  const int j = jb * kNodeJ + lane;
  const bool valid = wave == 0 && lane < kNodeJ && j < v.N;
  DPre p3{}, p5{}, p6{}, p7{};
  ZPre pn{};
  double yS = 0.0, nrm3 = 1.0, nrm5 = 1.0;
  if (valid) {
    p3 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o3 + j, copy_anchor);
    p5 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o5 + j, copy_anchor);
    if (v.has_n) {
      p6 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o6 + j, copy_anchor);
      p7 = dual_pre<INIT>(v, y, ya, kz, kza, dl.o7 + j, copy_anchor);
      pn = primal_pre(v, zi, zia, lb, ub, il.on + j, copy_anchor);
      if (v.step2) yS = y[dl.oS];
    }
    if (CHECK) {
      nrm3 = v.rownorm[dl.o3 + j];
      nrm5 = v.rownorm[dl.o5 + j];
    }
    const int pol_sw = first ? ctrl->polish_pending : 0;
    double *yb = v.ybak + slot * v.sdual;
    if (pol_sw == 1) {          // polishing starts: the node rows' duals kept, the feasibility problem's from 0
      yb[dl.o3 + j] = p3.y;
      yb[dl.o5 + j] = p5.y;
      if (v.has_n) {
        yb[dl.o6 + j] = p6.y;
        yb[dl.o7 + j] = p7.y;
      }
      p3.y = p5.y = p6.y = p7.y = 0.0;
      yS = 0.0;
    } else if (pol_sw == 2) {   // polishing ends uncertified: the kept duals come back
      if (v.step2) yS = yb[dl.oS];
      p3.y = yb[dl.o3 + j];
      p5.y = yb[dl.o5 + j];
      if (v.has_n) {
        p6.y = yb[dl.o6 + j];
        p7.y = yb[dl.o7 + j];
      }
    }
  }
  {
    const int jj = threadIdx.x % kNodeJ, g = threadIdx.x / kNodeJ;
    const int jl = jb * kNodeJ + jj;
    const int per = (F + NG - 1) / NG;
    const int f0 = g * per, f1 = min(F, f0 + per);
    double memc = 0.0, sumc = 0.0, U = 0.0, memr = 0.0, sumr = 0.0;
    if (jl < v.N) {
      const double *np_ = v.npart + slot * v.snpart;
      for (int f = f0; f < f1; ++f) {
        const double *p = np_ + (int64_t)f * 2 * NP;
        const double c = p[jl];
        memc += __dmul_rn(v.mem_f[f], c);   // the product x_pass used to store: same rounding, no FMA
        sumc += c;
        U += p[NP + jl];
      }
      if (CHECK) {
        const double *rp = v.rpart + slot * v.srpart;
        for (int f = f0; f < f1; ++f) {
          memr += rp[(int64_t)f * 2 * NP + jl];
          sumr += rp[(int64_t)f * 2 * NP + NP + jl];
        }
      }
    }
    red[0][g][jj] = memc;
    red[1][g][jj] = sumc;
    red[2][g][jj] = U;
    red[3][g][jj] = memr;
    red[4][g][jj] = sumr;
  }
  __syncthreads();
  if (wave != 0) return;
  // wave 0: fixed-order sums over the function groups
  double memc = 0.0, sumc = 0.0, U = 0.0, memr = 0.0, sumr = 0.0;
  if (lane < kNodeJ) {
#pragma unroll 8
    for (int g = 0; g < NG; ++g) {
      memc += red[0][g][lane];
      sumc += red[1][g][lane];
      U += red[2][g][lane];
      if (CHECK) {
        memr += red[3][g][lane];
        sumr += red[4][g][lane];
      }
    }
  }
  const double tau = INIT ? 0.0 : ctrl->tau, sigma = ctrl->sigma;
  const bool halp = !INIT && !plain;
  const double lam = halpern_lambda(ctrl, halp, it);
  float *kty = v.kty + slot * v.skty;
  SmallAcc a;
  double score_n = 0.0, score_n_rep = 0.0;
  if (valid && CHECK) {
    // certificate point (see x_pass): C3 at the repaired c, C5 (x only)
    a.res = fmax(a.res, row_viol(memr, p3.lo, p3.hi) / nrm3);
    a.res = fmax(a.res, row_viol(U, p5.lo, p5.hi) / nrm5);
    // the node rows' and n's bound terms at the repaired duals (C6/C7 at node j's price t*: the same
    // t* x_pass priced c with, from the same pre-update duals; DESIGN.md §4 "Dual repair")
    a.lagrR += row_lagr(p3.y, p3.lo, p3.hi) + row_lagr(p5.y, p5.lo, p5.hi);
    if (v.has_n) {
      const double bn = node_base(v, y, j);
      const double ts = repair_node(v, p6.y + p7.y, bn, pn.z, pn.lb, pn.ub);
      const double rcn = price_rc(bn, ts, v.M);
      a.lagrR += row_lagr(fmin(ts, 0.0), p6.lo, p6.hi) + row_lagr(fmax(ts, 0.0), p7.lo, p7.hi) +
                 fmin(pn.lb * rcn, pn.ub * rcn);
    }
  }
  if (valid) {
    dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o3 + j, memc, p3, sigma, copy_anchor, halp, lam, a);
    const double y5n = dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o5 + j, U, p5, sigma, copy_anchor, halp, lam, a);
    kty[(int64_t)F * NP + j] = (float)y5n;
    if (v.has_n) {
      const double kty_n = -v.M * p6.y - p7.y + v.score_n_coef * yS;
      const double ncost = ctrl->polish ? 0.0 : pn.cost;   // polishing: objective off (the certificate keeps it)
      const double nn = primal_step_p<CHECK>(zi, zia, il.on + j, ncost - kty_n, pn, tau, copy_anchor, halp, lam, a);
      dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o6 + j, sumc - v.M * nn, p6, sigma, copy_anchor, halp, lam, a);
      dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.o7 + j, sumc - nn, p7, sigma, copy_anchor, halp, lam, a);
      score_n = v.score_n_coef * nn;
      if (CHECK) {
        // repaired n: the T output clamped into [sum c / M, sum c + eps] (C6/C7 at the repaired c)
        const double lon = fmax(pn.lb, sumr / v.M), hin = fmin(pn.ub, sumr + v.eps);
        const double nr = lon > hin ? lon : fmin(fmax(nn, lon), hin);
        a.res = fmax(a.res, lon - hin);
        a.pobj += pn.cost * nr;
        v.zr[slot * v.sint + il.on + j] = nr;
        score_n_rep = v.score_n_coef * nr;
      }
    }
  }
  // the node blocks' scalar partials: read by scalar_pass on init / certificate iterations, and for the
  // step-2 score row on every step-2 iteration (plain step-1 iterations skip 21 wave reductions)
  if (CHECK || INIT) write_bpart<true>(v.bpart + slot * v.sbpart + ((int64_t)F + jb) * NBS, a, 0.0, score_n, score_n_rep, lane);
  else if (v.step2) write_bpart<false>(v.bpart + slot * v.sbpart + ((int64_t)F + jb) * NBS, a, 0.0, score_n, score_n_rep, lane);
}

// Primal feasibility polishing (scalar_pass): after nep_lp_opts.polish_after iterations, an LP whose best
// Lagrangian bound is within half the gap tolerance of its repaired point's objective and whose
// primal residual is in (tol, kPolishRes] switches to its feasibility problem.
// (kPolishRes / kPolishBudget: nep_internal.h; NEP_POLISH="res,budget" overrides them)

// ---------------------------------------------------------------------------------------------
// scalar_pass: one workgroup per slot.  Step-2 scalar rows (D3a, D3b, D4, score) and the
// integer-bounded a / d variables; at check iterations the certificate (primal objective,
// Lagrangian bound, residuals), status, restarts and the primal-weight update.
// ---------------------------------------------------------------------------------------------
template <bool CHECK, bool INIT>
__global__ __launch_bounds__(256) void scalar_pass(DeviceView v, const int32_t *__restrict__ slots, int first,
                                                   int plain, int it, int block_len) {
  __shared__ double tot[NTS + NBS];
  const int slot = slots[blockIdx.x];
  Ctrl *ctrl = v.ctrl + slot;
  if (!ctrl->active) return;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1), wave = tid >> 6;
  const double *tp = v.tpart + slot * v.stpart;
  const double *bp = v.bpart + slot * v.sbpart;
  const int nb = v.F + v.JB;
  // deterministic reductions of the partials (fixed per-lane order, fixed wave tree): the fields are
  // dealt over the 4 waves, one wave reduces a field alone (no block-wide tree per field).  Plain
  // step-2 iterations need only the fields of the step-2 rows (sum c, the score row).
  for (int k = wave; k < NTS + NBS; k += 4) {
    const bool needed = CHECK || INIT || k == TS_SCORE || k == NTS + BS_SUMC_NEW || k == NTS + BS_SCORE_N;
    if (!needed) {
      if (lane == 0) tot[k] = 0.0;
      continue;
    }
    const bool is_max = (k == NTS + BS_RES);
    double acc = 0.0;
    if (k < NTS) {
      for (int t = lane; t < v.F; t += kWave) acc += tp[(int64_t)t * NTS + k];
    } else {
      for (int t = lane; t < nb; t += kWave) {
        const double u = bp[(int64_t)t * NBS + (k - NTS)];
        acc = is_max ? fmax(acc, u) : acc + u;
      }
    }
    acc = is_max ? wave_max_d(acc) : wave_sum_d(acc);
    if (lane == 0) tot[k] = acc;
  }
  __syncthreads();
  // step-2 certificate: G(lambda_q) = min over (a, d, T) of ca a + cd d + lambda_q T on the boxes and
  // the rows D3a/D3b/D4, by its vertices (3 of at most 12 half-spaces g . (a, d, T) >= h: 220
  // triples, one per thread).  A vertex is accepted within 1e-9 of every half-space: accepting a
  // slightly infeasible one can only lower the minimum, so the bound stays valid.
  __shared__ double gmin[kNLam][256];
  if (CHECK && v.step2 && !v.dred) {
    const DualLayout &dl = v.dl;
    const IntLayout &il = v.il;
    const double *lbs = v.lb + slot * v.sint, *ubs = v.ub + slot * v.sint;
    double lamk[kNLam];
    dblock_lambdas(v, v.y + slot * v.sdual, lamk);
    double hg[12][3], hh[12];
    int nh = 0;
    auto add = [&](double ga, double gd, double gt, double h) {
      if (!isfinite(h)) return;
      hg[nh][0] = ga; hg[nh][1] = gd; hg[nh][2] = gt; hh[nh] = h; ++nh;
    };
    add(1, 0, 0, lbs[il.oa]);  add(-1, 0, 0, -ubs[il.oa]);
    add(0, 1, 0, lbs[il.od]);  add(0, -1, 0, -ubs[il.od]);
    add(0, 0, 1, tot[NTS + BS_TLO]);  add(0, 0, -1, -tot[NTS + BS_THI]);
    const int rws[3] = {dl.oD3a, dl.oD3b, dl.oD4};
    const double rg[3][3] = {{-1, 0, -1}, {0, -1, 1}, {1, 1, v.sigma4}};
    for (int q = 0; q < 3; ++q) {
      add(rg[q][0], rg[q][1], rg[q][2], v.lo[rws[q]]);
      add(-rg[q][0], -rg[q][1], -rg[q][2], -v.hi[rws[q]]);
    }
    const double ca = v.cost_int[il.oa], cd = v.cost_int[il.od];
    double best[kNLam];
#pragma unroll
    for (int q = 0; q < kNLam; ++q) best[q] = INFINITY;
    int t = 0;
    for (int i0 = 0; i0 < nh; ++i0)
      for (int i1 = i0 + 1; i1 < nh; ++i1)
        for (int i2 = i1 + 1; i2 < nh; ++i2, ++t) {
          if ((t & 255) != tid) continue;
          const double *g0 = hg[i0], *g1 = hg[i1], *g2 = hg[i2];
          const double det = g0[0] * (g1[1] * g2[2] - g1[2] * g2[1]) - g0[1] * (g1[0] * g2[2] - g1[2] * g2[0]) +
                             g0[2] * (g1[0] * g2[1] - g1[1] * g2[0]);
          if (fabs(det) < 1e-12) continue;
          const double h0 = hh[i0], h1 = hh[i1], h2 = hh[i2];
          const double va = (h0 * (g1[1] * g2[2] - g1[2] * g2[1]) - g0[1] * (h1 * g2[2] - g1[2] * h2) +
                             g0[2] * (h1 * g2[1] - g1[1] * h2)) / det;
          const double vd = (g0[0] * (h1 * g2[2] - g1[2] * h2) - h0 * (g1[0] * g2[2] - g1[2] * g2[0]) +
                             g0[2] * (g1[0] * h2 - h1 * g2[0])) / det;
          const double vt = (g0[0] * (g1[1] * h2 - h1 * g2[1]) - g0[1] * (g1[0] * h2 - h1 * g2[0]) +
                             h0 * (g1[0] * g2[1] - g1[1] * g2[0])) / det;
          bool ok = true;
          for (int e = 0; e < nh; ++e)
            ok = ok && (hg[e][0] * va + hg[e][1] * vd + hg[e][2] * vt >= hh[e] - 1e-9 * (1.0 + fabs(hh[e])));
          if (!ok) continue;
#pragma unroll
          for (int q = 0; q < kNLam; ++q) best[q] = fmin(best[q], ca * va + cd * vd + lamk[q] * vt);
        }
#pragma unroll
    for (int q = 0; q < kNLam; ++q) gmin[q][tid] = best[q];
    __syncthreads();
    for (int s2 = 128; s2 > 0; s2 >>= 1) {
      if (tid < s2) {
#pragma unroll
        for (int q = 0; q < kNLam; ++q) gmin[q][tid] = fmin(gmin[q][tid], gmin[q][tid + s2]);
      }
      __syncthreads();
    }
  }
  // the slot's certificate, status and restart decisions: thread 0 (a lambda, so that every thread
  // meets the barrier below); a polished LP that certifies gets its kept duals back (restore_duals)
  __shared__ int restore_duals;
  if (tid == 0) restore_duals = 0;
  if (tid == 0) [&]() {

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
  a.lagrD = tot[NTS + BS_LAGR_D];
  double score_lagr = 0.0;   // the step-2 score row's bound term (pre-update dual)
  double dred_lagr = 0.0;    // reduced step 2: the row sum c's bound term (pre-update dual)

  if (v.step2) {
    const double sumc = tot[NTS + BS_SUMC_NEW];
    const double score = tot[TS_SCORE] + tot[NTS + BS_SCORE_N];
    double yD3a = y[dl.oD3a], yD3b = y[dl.oD3b], yD4 = y[dl.oD4], yS = y[dl.oS];
    // polishing: these rows' duals are kept / restarted from 0 / read back like the others
    const int pol_sw = first ? ctrl->polish_pending : 0;
    double *yb = v.ybak + slot * v.sdual;
    if (pol_sw == 1) {
      yb[dl.oD3a] = yD3a; yb[dl.oD3b] = yD3b; yb[dl.oD4] = yD4; yb[dl.oS] = yS;
      yD3a = yD3b = yD4 = yS = 0.0;
    } else if (pol_sw == 2) {
      yD3a = yb[dl.oD3a]; yD3b = yb[dl.oD3b]; yD4 = yb[dl.oD4]; yS = yb[dl.oS];
    }
    const double csd = ctrl->polish ? 0.0 : 1.0;
    if (v.dred) {
      // reduced disruption block: the row sum c in [L, U] (D4's dual; dred_interval), a / d not iterated
      double L, U;
      dred_bounds(v, lb, ub, L, U);
      if (CHECK) dred_lagr = row_lagr(yD4, L, U);
      DPre p = dual_pre<INIT>(v, y, ya, kz, kza, dl.oD4, copy_anchor);
      p.y = yD4;
      p.lo = L;
      p.hi = U;
      dual_step_p<CHECK, INIT>(y, ya, kz, kza, dl.oD4, sumc, p, sigma, copy_anchor, halp, lam, a);
    } else {
    // allocated (a): D3a coef -1, D4 coef +1 ; deallocated (d): D3b coef -1, D4 coef +1
    const double an = primal_step<CHECK>(v, zi, zia, lb, ub, il.oa, csd * v.cost_int[il.oa] - (-yD3a + yD4), tau,
                                         copy_anchor, halp, lam, a, true);
    const double dn = primal_step<CHECK>(v, zi, zia, lb, ub, il.od, csd * v.cost_int[il.od] - (-yD3b + yD4), tau,
                                         copy_anchor, halp, lam, a, true);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD3a, -sumc - an, yD3a, sigma, copy_anchor, halp, lam, a, true);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD3b, sumc - dn, yD3b, sigma, copy_anchor, halp, lam, a, true);
    dual_step<CHECK, INIT>(v, y, ya, kz, kza, dl.oD4, dn + an + v.sigma4 * sumc, yD4, sigma, copy_anchor, halp, lam,
                           a, true);
    }
    if (CHECK) score_lagr = row_lagr(yS, v.lo[dl.oS], v.hi[dl.oS]);
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

  // iterations since the last certificate: 1 at the slot's first certificate (its first
  // iteration), a whole block afterwards — per slot, so slots may join between blocks
  const int64_t done = ctrl->k == 0 ? 1 : block_len;
  ctrl->k += done;
  ctrl->k_lineage += done;
  ctrl->k_since_restart += done;
  ctrl->restart_pending = 0;
  ctrl->polish_pending = 0;
  if (tot[TS_EMPTY] > 0) { ctrl->status = 2; ctrl->active = 0; return; }
  // certificate point, completed: allocated / deallocated repaired from the repaired sum c
  // (D3: a <= sumOld - sum c, d <= sum c - sumOld; D4: a + d >= sigma4 (sumOld - sum c); costs
  // (w-1) a + (w+1) d, both positive: a as large as allowed, d = the rest), the score row at the
  // repaired n.  Its objective is an upper bound on the LP value whenever it is feasible (res <= tol),
  // the Lagrangian a lower bound: the gap between the two certifies the node LP's value.
  double pobj = a.pobj, res = a.res;   // x part (TS_POBJ) + repaired small variables
  if (v.step2) {
    const double sum_old = v.lo[dl.oD3b];
    const double s = tot[NTS + BS_SUMC_REP] - sum_old;
    const double A = fmin(ub[il.oa], -s), Dm = fmin(ub[il.od], s), K = v.sigma4 * (-s);
    const double ar = fmax(lb[il.oa], A);
    const double dr = fmax(lb[il.od], K - ar);
    res = fmax(res, fmax(lb[il.oa] - A, dr - Dm));
    pobj += v.cost_int[il.oa] * ar + v.cost_int[il.od] * dr;
    v.zr[slot * v.sint + il.oa] = ar;
    v.zr[slot * v.sint + il.od] = dr;
    if (v.dred) { zi[il.oa] = ar; zi[il.od] = dr; }   // (not iterated: the last certificate's values)
    const double score_rep = tot[TS_SCORE] + tot[NTS + BS_SCORE_N_REP];
    res = fmax(res, row_viol(score_rep, v.lo[dl.oS], v.hi[dl.oS]) / v.rownorm[dl.oS]);
  }
  // the Lagrangian with every row dualised, or (step 2) the disruption block kept exact at the best
  // of the candidate prices (both are valid bounds)
  double lagr = a.lagr + a.lagrD;
  // reduced step 2: the block's constant -sT sum old (the (f, j) constants are in a.lagr: x_pass)
  const double dred_k0 = (v.dred && !ctrl->polish) ? -v.sT * v.sum_old : 0.0;
  lagr += dred_k0;
  // Infeasibility (Farkas): with the objective off the Lagrangian L0(y) is positively
  // homogeneous in y and <= 0 at every y when the LP has a feasible point; L0(y) > 0 at a sign-feasible
  // y proves the node LP infeasible (L(t y) >= t L0(y) + min cost -> +inf).  The margin is far above the
  // fp64 rounding of the sums.  (Not while polishing: its passes carry no cost in rc.)
  const double lagr0 = tot[TS_LAGR0] + tot[NTS + BS_LAGR0] + a.lagr0;
  // (two consecutive checks: the duals of an infeasible LP keep running off along the ray, so the test
  // keeps holding; a one-off from rounding in the sums does not)
  if (!ctrl->polish && isfinite(lagr0) && lagr0 > 1e-6 * fmax(1.0, fabs(lagr))) {
    if (++ctrl->infeas_hits >= 2) { ctrl->status = 2; ctrl->active = 0; ctrl->lagr = INFINITY; return; }
  } else {
    ctrl->infeas_hits = 0;
  }
  if (v.step2 && !v.dred) {
#pragma unroll
    for (int q = 0; q < kNLam; ++q)
      if (isfinite(gmin[q][0])) lagr = fmax(lagr, a.lagr + tot[NTS + BS_LK0 + q] + gmin[q][0]);
  }
  // ... and the same bound at the repaired duals (DESIGN.md §4 "Dual repair"): the larger one stands
  if (!v.fac) {   // (the facility relaxation has no big-M pairs to repair)
    double lr = tot[TS_LAGR_REP] + tot[NTS + BS_LAGR_REP];
    if (v.dred) {
      lr += score_lagr + dred_lagr + dred_k0;
    } else if (v.step2) {
      double best = -INFINITY;
#pragma unroll
      for (int q = 0; q < kNLam; ++q)
        if (isfinite(gmin[q][0])) best = fmax(best, tot[NTS + BS_LKR0 + q] + gmin[q][0]);
      lr += score_lagr + best;
    }
    if (lr > lagr) lagr = lr;
  }
  const double gap = pobj - lagr;
  const double tol = v.prm[0], cutoff = v.prm[1], gap_tol = v.prm[2];
  ctrl->pobj = pobj;
  // An exact LP (below) has the value pobj if it is feasible at all, so pobj bounds it from below
  // whether or not this point is feasible yet (an infeasible LP has value +inf): a leaf whose fixed
  // placement costs more than the incumbent is cut off at its first check instead of iterating on to
  // feasibility.
  if (ctrl->exact && isfinite(pobj)) ctrl->best_lagr = fmax(ctrl->best_lagr, pobj);
  if (ctrl->exact && isfinite(pobj) && res <= tol) {
    // The node box fixes every variable that carries cost (a leaf of a model whose routing has no
    // cost: step 2, or W == 0): every feasible point has the repaired point's objective, so a
    // feasible repaired point IS an LP optimum and its objective the LP value.
    ctrl->lagr = pobj;
    ctrl->best_lagr = fmax(ctrl->best_lagr, pobj);
    ctrl->pres = res;
    ctrl->gap = 0.0;
    ctrl->status = 0;
    ctrl->active = 0;
    return;
  }
  if (ctrl->polish) {
    // Polishing: the iterate solves the feasibility problem, whose Lagrangian bounds nothing here.
    // The bound is the best one taken before polishing; the repaired point's objective (reference
    // costs) is measured against it.
    const double b = ctrl->polish_bound;
    ctrl->lagr = b;
    ctrl->pres = res;
    ctrl->gap = pobj - b;
    if (res <= tol && pobj - b <= gap_tol * fmax(1.0, fabs(b))) {
      ctrl->status = 0;
      ctrl->active = 0;
      restore_duals = 1;
      return;
    }
    if (ctrl->bound_res > 0.0 && res <= ctrl->bound_res && pobj - b <= gap_tol * fmax(1.0, fabs(b))) {   // B&B node
      ctrl->status = 5;   // NEP_LP_BOUND
      ctrl->active = 0;
      restore_duals = 1;
      return;
    }
  } else {
    ctrl->lagr = lagr;
    if (lagr > ctrl->best_lagr) ctrl->best_lagr = lagr;
    ctrl->pres = res;
    ctrl->gap = gap;
    // certified against the best bound seen so far (every Lagrangian bound of this LP is valid, the
    // repaired point is this iteration's): the value reported is that bound
    const double bl = ctrl->best_lagr;
    if (isfinite(bl) && res <= tol && pobj - bl <= gap_tol * fmax(1.0, fabs(bl))) {
      ctrl->lagr = bl;
      ctrl->gap = pobj - bl;
      ctrl->status = 0; ctrl->active = 0; return;
    }
    // a B&B node's bound has converged (nep_lp_opts.bound_res): its residual need not reach tol, since
    // the node branches on the bound, which is valid at any dual point
    if (ctrl->bound_res > 0.0 && isfinite(bl) && res <= ctrl->bound_res && pobj - bl <= gap_tol * fmax(1.0, fabs(bl))) {
      ctrl->status = 5; ctrl->active = 0; return;   // NEP_LP_BOUND
    }
  }
  if (ctrl->best_lagr > cutoff) { ctrl->status = 3; ctrl->active = 0; return; }
  if (ctrl->k >= ctrl->max_iters) { ctrl->status = 1; ctrl->active = 0; return; }
  if (!isfinite(pobj) || !isfinite(a.mvz) || !isfinite(a.mvy)) { ctrl->status = 4; ctrl->active = 0; return; }

  // primal feasibility polishing (step 1 and step 2; the step-2 duals D1/D2 are kept by x_pass, D3a/D3b/
  // D4/score by this pass): the best bound already meets the gap test against the
  // repaired point's objective and only its primal residual is left — the tail of the node LPs,
  // whose CPU rows (C5) close last (tools/probes/tail_probe.py).  From here the LP iterates on its
  // feasibility problem (objective off, duals restarted from 0) from the current point; it is
  // certified once the repaired point is feasible within tol and its objective still within the
  // gap tolerance of the bound kept.
  bool polish_now = false;
  if (ctrl->polish) {
    if (ctrl->k - ctrl->polish_k0 >= v.polish_budget) {   // not certified within the budget: back to the LP
      ctrl->polish = 0;
      ctrl->polish_pending = 2;
      ctrl->polish_next = ctrl->k + 4 * v.polish_budget;
      polish_now = true;                                 // (restart: the anchors take the restored duals)
    }
  } else if (ctrl->polish_next >= 0 && ctrl->k >= ctrl->polish_next && res > tol && res <= v.polish_res &&
             isfinite(ctrl->best_lagr) &&
             fabs(pobj - ctrl->best_lagr) <= 0.5 * gap_tol * fmax(1.0, fabs(ctrl->best_lagr))) {
    ctrl->polish = 1;
    ctrl->polish_pending = 1;   // consumed by the passes of the block's next iteration (it == 1)
    ctrl->polish_bound = ctrl->best_lagr;
    ctrl->polish_k0 = ctrl->k;
    polish_now = true;
  }
  // restart test on the fixed-point residual of the last iteration (ω-weighted norm)
  const double w = ctrl->omega;
  const double fpr = sqrt(w * a.mvz + a.mvy / w);
  if (ctrl->last_restart_fpr < 0) ctrl->last_restart_fpr = fpr;
  const bool restart = polish_now || (fpr <= v.rs_suff * ctrl->last_restart_fpr) ||
                       (fpr <= v.rs_nec * ctrl->last_restart_fpr && fpr > ctrl->prev_fpr) ||
                       (ctrl->k_since_restart >= v.rs_art * ctrl->k);
  ctrl->prev_fpr = fpr;
  if (restart) {
    const double dz = sqrt(a.dsz), dy = sqrt(a.dsy);
    if (!polish_now && dz > 1e-10 && dy > 1e-10) {   // (entering polishing keeps the weight)
      double nw = exp(v.omega_smooth * log(dy / dz) + (1.0 - v.omega_smooth) * log(w));
      nw = fmin(fmax(nw, ctrl->omega_lo), ctrl->omega_hi);
      ctrl->omega = nw;
      ctrl->tau = ctrl->eta / nw;
      ctrl->sigma = ctrl->eta * nw;
    } else if (!polish_now && v.dred && dz <= 1e-10 && dy > 1e-10) {
      // reduced step 2: the primal has not moved since the last restart while the dual has — the weight is so
      // small that every primal step lands on the same box corner (the PDLP ratio dy / dz is +inf): raise it
      // 10x (numpy mirror, small step-2 goldens at the reduced LP's initial weight: payload.json model 1 stalled
      // at 60k iterations with the primal static, certifies in 1217 with this rule)
      const double nw = fmin(w * 10.0, ctrl->omega_hi);
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
  }();
  // (also when a polishing LP stops uncertified: its bound is the kept one, its state the LP's duals)
  if (tid == 0 && ctrl->polish && !ctrl->active) restore_duals = 1;
  __syncthreads();
  if (restore_duals) {
    // The certified point is the polished primal; its dual state goes back to the LP's own duals (kept
    // when polishing started), so children warm-started from this slot start from them, not from
    // the feasibility problem's.
    double *y = v.y + slot * v.sdual;
    const double *yb = v.ybak + slot * v.sdual;
    for (int i = tid; i < v.dl.n_dual; i += 256) y[i] = yb[i];
  }
}

// cold / warm initialisation of a slot (x̄ ← 0 for cold; the init passes project it)
__global__ void init_slot(DeviceView v, const int32_t *__restrict__ slots, const int32_t *__restrict__ exact, int warm,
                          double eta, double omega0, const double *__restrict__ per) {
  const int slot = slots[blockIdx.y];
  Ctrl *ctrl = v.ctrl + slot;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double *zi = v.zi + slot * v.sint;
  const double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  if (!warm) {
    float *x = v.x + slot * v.sx;
    for (int64_t i = tid; i < (int64_t)v.R * v.NP; i += stride) x[i] = 0.f;
    if (v.fac) {   // the x <= c duals and their sums
      float *lam = v.lam + slot * v.sx, *ls = v.lsum + slot * v.slsum;
      for (int64_t i = tid; i < (int64_t)v.R * v.NP; i += stride) lam[i] = 0.f;
      for (int64_t i = tid; i < v.slsum; i += stride) ls[i] = 0.f;
    }
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
    // A warm-started child keeps its parent's primal weight as a floor (times warm_omega_floor):
    // the PDLP update right after a warm start sees the large primal move of re-routing the fixed
    // placements and would shrink omega by orders of magnitude, which stalls the dual (measured on
    // the 512x256 bench children: 81/96 certified within 20k iterations without a floor, 95/96 with
    // floor 2, 62k iterations in all instead of 304k; tools/probes/floor_probe.py).
    if (warm && v.warm_omega_floor > 0) ctrl->omega_lo = fmin(ctrl->omega * v.warm_omega_floor, ctrl->omega_hi);
    // ... and, once that weight has been adapted over kOmegaTrained iterations of its lineage, at most
    // warm_omega_cap times it: without a cap the first restart after a warm start can raise it 50x on
    // the dual's large move toward the fixings, and the child then stalls at the node-LP limit (512x256
    // bench seed 0: 39/128 children certified, 125/128 with cap 4).  A weight that never
    // adapted (a root certified in a few iterations) is left free.
    if (!warm) ctrl->k_lineage = 0;
    if (warm && v.warm_omega_cap > 0 && ctrl->k_lineage >= kOmegaTrained)
      ctrl->omega_hi = fmax(ctrl->omega * v.warm_omega_cap, ctrl->omega_lo);
    // With a model reference weight (nep_lp_set_reference_weight) the band is [floor, cap] x that reference and
    // the parent's weight is clamped into it: relative to the parent, the band ratchets up along a lineage of
    // warm starts (512x256 replay: uncertified node LPs at a median 80x the root's weight; 8.8 -> 11.4
    // certified LP/s with the band fixed; DESIGN.md §4 "Warm-start primal weight")
    if (warm && v.warm_omega_ref > 0) {
      ctrl->omega_lo = v.warm_omega_floor > 0 ? v.warm_omega_ref * v.warm_omega_floor : omega0 * 1e-5;
      ctrl->omega_hi = fmax(v.warm_omega_cap > 0 ? v.warm_omega_ref * v.warm_omega_cap : omega0 * 1e5, ctrl->omega_lo);
      ctrl->omega = fmin(fmax(ctrl->omega, ctrl->omega_lo), ctrl->omega_hi);
    }
    ctrl->tau = eta / ctrl->omega;
    ctrl->sigma = eta * ctrl->omega;
    ctrl->status = 1;
    ctrl->active = 1;
    ctrl->exact = exact[blockIdx.y];
    // (nep_lp_submit_ex: per-LP iteration budget and bound stop, per = [2][nslots]; else the call's)
    ctrl->max_iters = per ? (int64_t)per[blockIdx.y] : v.max_iters;
    ctrl->bound_res = per ? per[gridDim.y + blockIdx.y] : v.bound_res;
    ctrl->infeas_hits = 0;
    ctrl->restart_pending = 1;
    ctrl->polish = ctrl->polish_pending = 0;   // a warm start does not inherit its parent's polishing
    ctrl->polish_bound = -INFINITY;
    ctrl->polish_k0 = 0;
    ctrl->polish_next = v.polish_after;   // this LP's submit option (-1: it never polishes)
    ctrl->best_lagr = -INFINITY;
    ctrl->pobj = ctrl->lagr = ctrl->pres = ctrl->gap = NAN;
  }
}

// a node's box on the device: the model's base box (natural bounds, all allowed destinations) ...
__global__ void node_bounds_base(DeviceView v, const int32_t *__restrict__ slots, const double *__restrict__ blb,
                                 const double *__restrict__ bub, const uint8_t *__restrict__ bmask) {
  const int slot = slots[blockIdx.y];
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  for (int64_t i = tid; i < v.sint; i += stride) {
    lb[i] = blb[i];
    ub[i] = bub[i];
  }
  uint8_t *mask = v.mask + slot * v.smask;
  for (int64_t i = tid; i < v.smask; i += stride) mask[i] = bmask[i];
}
// ... then the node's packed bound changes (presolve_node, nep_host.cpp), with the destination
// masks of the changed c[f, j]
__global__ void node_bounds_scatter(DeviceView v, const int32_t *__restrict__ slots, const int32_t *__restrict__ off,
                                    const int32_t *__restrict__ idx, const double *__restrict__ cl,
                                    const double *__restrict__ cu) {
  const int b = blockIdx.y;
  const int slot = slots[b];
  double *lb = v.lb + slot * v.sint, *ub = v.ub + slot * v.sint;
  uint8_t *mask = v.mask + slot * v.smask;
  const int oc = v.il.oc, FN = v.F * v.N;
  for (int t = off[b] + blockIdx.x * blockDim.x + threadIdx.x; t < off[b + 1]; t += gridDim.x * blockDim.x) {
    const int k = idx[t];
    lb[k] = cl[t];
    ub[k] = cu[t];
    if (k >= oc && k < oc + FN) {
      const int f = (k - oc) / v.N, j = (k - oc) - f * v.N;
      mask[(int64_t)f * v.NP + j] = cu[t] > 0.0 ? 1 : 0;
    }
  }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int CPL, int TW>
static hipError_t launch_x_tw(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                              bool first, bool plain, int it, hipStream_t s) {
  dim3 grid(8 * ((v.F * nslots + 7) / 8)), block(kWave * TW);
  const size_t lds = (size_t)(2 * TW + 2) * v.NP * sizeof(float) +
                    (check ? (size_t)(NEP_INLINE_REFLECT ? 3 : 2) * TW * v.NP * sizeof(float) + 4 * v.NP * sizeof(double) : 0);
  const int pl = plain ? 1 : 0;
  // non-temporal routing streams only when the iterating slots' x + anchor exceed ~160 MB (see ld_x4)
  const int nt = (double)nslots * 2.0 * (double)v.sx * sizeof(float) > 160e6 ? 1 : 0;
  if (init) hipLaunchKernelGGL((x_pass<CPL, false, true, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else if (check)
    hipLaunchKernelGGL((x_pass<CPL, true, false, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else if (first)
    hipLaunchKernelGGL((x_pass<CPL, false, false, true, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  else hipLaunchKernelGGL((x_pass<CPL, false, false, false, TW>), grid, block, lds, s, v, slots, pl, it, nslots, nt);
  return hipGetLastError();
}

// Waves per workgroup: 4 when the LP slots alone fill the chip, more when few slots iterate (the
// root LP, the tail of a B&B batch), so every CU still holds >= 16 waves: one LP at 512x256 runs
// its x pass 1.9x faster with 16 waves (root LP 7.3 s -> 3.9 s) while 4 waves stay fastest from
// ~4 slots on (0.47 vs 0.57 ms per launch at ~15 slots).  The column sums are then added in another
// (still fixed) order, so an LP's last bits depend on how many slots iterated beside it.
// Only the certificate variant is held to 144 KB of LDS (fp64 column / CPU sums + constants: fp32, fp64,
// repaired prices, pooled flow), i.e. to 8 waves at N = 512; the plain iterations of a lone root keep
// 16 (2 x 16 x N fp32 accumulators: 66 KB at N = 512).
static int tile_waves(const DeviceView &v, int nslots, bool check) {
  int tw = 4;
  while (tw < 16 && (int64_t)nslots * v.F * tw < 4096) tw *= 2;
  if (v.CPL >= 8 && tw > 8) tw = 8;   // (N > 1024: 1024-thread workgroups cap a lane at 128 VGPRs, which spill)
  while (check && tw > 4 && (size_t)((NEP_INLINE_REFLECT ? 5 : 4) * tw + 2) * v.NP * sizeof(float) + 4 * v.NP * sizeof(double) > 144 * 1024)
    tw /= 2;
  return tw;
}

template <int CPL>
static hipError_t launch_x_cpl(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                               bool first, bool plain, int it, hipStream_t s) {
  switch (tile_waves(v, nslots, check)) {
    case 4: return launch_x_tw<CPL, 4>(v, slots, nslots, check, init, first, plain, it, s);
    case 8: return launch_x_tw<CPL, 8>(v, slots, nslots, check, init, first, plain, it, s);
    case 16: return launch_x_tw<CPL, 16>(v, slots, nslots, check, init, first, plain, it, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fac_x_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                             bool plain, int it, hipStream_t s);
hipError_t launch_fac_node_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                                bool plain, int it, hipStream_t s);

hipError_t launch_x_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                         bool plain, int it, hipStream_t s) {
  if (v.fac) return launch_fac_x_pass(v, slots, nslots, check, init, first, plain, it, s);   // (nep_fac.hip)
  switch (v.CPL) {
    case 1: return launch_x_cpl<1>(v, slots, nslots, check, init, first, plain, it, s);
    case 2: return launch_x_cpl<2>(v, slots, nslots, check, init, first, plain, it, s);
    case 4: return launch_x_cpl<4>(v, slots, nslots, check, init, first, plain, it, s);
    case 8: return launch_x_cpl<8>(v, slots, nslots, check, init, first, plain, it, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_node_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                            bool plain, int it, hipStream_t s) {
  if (v.fac) return launch_fac_node_pass(v, slots, nslots, check, init, first, plain, it, s);
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  dim3 grid(v.JB, nslots), block(kNodeThreads);   // JB = ceil(N / kNodeJ)
  if (init) hipLaunchKernelGGL((node_pass<false, true>), grid, block, 0, s, v, slots, fi, pl, it);
  else if (check) hipLaunchKernelGGL((node_pass<true, false>), grid, block, 0, s, v, slots, fi, pl, it);
  else hipLaunchKernelGGL((node_pass<false, false>), grid, block, 0, s, v, slots, fi, pl, it);
  return hipGetLastError();
}

hipError_t launch_scalar_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                              bool first, bool plain, int it, int block_len, hipStream_t s) {
  dim3 grid(nslots), block(256);
  const int fi = first ? 1 : 0, pl = plain ? 1 : 0;
  if (init)
    hipLaunchKernelGGL((scalar_pass<false, true>), grid, block, 0, s, v, slots, fi, pl, it, block_len);
  else if (check)
    hipLaunchKernelGGL((scalar_pass<true, false>), grid, block, 0, s, v, slots, fi, pl, it, block_len);
  else
    hipLaunchKernelGGL((scalar_pass<false, false>), grid, block, 0, s, v, slots, fi, pl, it, block_len);
  return hipGetLastError();
}

hipError_t launch_node_bounds(const DeviceView &v, const int32_t *slots, int nslots, const double *base_lb,
                              const double *base_ub, const uint8_t *base_mask, const int32_t *off, const int32_t *idx,
                              const double *cl, const double *cu, int max_chg, hipStream_t s) {
  hipLaunchKernelGGL(node_bounds_base, dim3(128, nslots), dim3(256), 0, s, v, slots, base_lb, base_ub, base_mask);
  if (max_chg > 0) {
    const int gx = std::min(64, (max_chg + 255) / 256);
    hipLaunchKernelGGL(node_bounds_scatter, dim3(gx, nslots), dim3(256), 0, s, v, slots, off, idx, cl, cu);
  }
  return hipGetLastError();
}

hipError_t launch_init_slot(const DeviceView &v, const int32_t *slots, const int32_t *exact, int nslots, bool warm,
                            double eta, double omega0, const double *per, hipStream_t s) {
  dim3 grid(256, nslots), block(256);
  hipLaunchKernelGGL(init_slot, grid, block, 0, s, v, slots, exact, warm ? 1 : 0, eta, omega0, per);
  return hipGetLastError();
}

}  // namespace nep
