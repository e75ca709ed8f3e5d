// nep_internal.h — shared host/device layout of the NEPTUNE LP engine (MI355X / gfx950).
//
// One model = one structured LP family (a reference step model, neptune_step1.py / neptune_step2.py)
// and `max_batch` LP slots (B&B nodes).  Layout in HBM (per slot unless noted):
//
//   x     [R][NP] f32   routing rows x̄[r, j]; row r = (function f, source i) or the pooled
//                       zero-workload sources of f (exact aggregation); the rows of
//                       one function are consecutive (frow[f] .. frow[f+1])
//   xa    [R][NP] f32   restart anchor of x, dense form (only rows whose anchor has > kAnchorK nonzeros)
//   acnt  [R] i32       anchor nonzeros of each row (kAnchorDense: the row's anchor is dense in xa)
//   aent  [R][kAnchorK] (j, value) pairs of the anchor rows held sparse
//   mask  [F][NP] u8    destination j allowed for function f at this node (c_ub[f,j] > 0)
//   zi    [n_int] f64   small primal: c, (mf, mt, a, d), n        + anchor zia, bounds lb/ub
//   y     [n_dual] f64  duals of the dualised rows   + anchor ya, activity kz (iterate) / kza (anchor) (built with
//                       NEP_INLINE_REFLECT, C1/C2/D1/D2 reflect in x_pass and leave theirs unused)
//   kty   [F*NP + NP + 4] f32  packed duals the x pass needs: y1+y2 per (f,j), y5 per j, yS
//   tpart [F][NTS] f64  per-function scalars of the rows (score row, objective, Lagrangian, movement)
//   npart [F][2][NP] f64 per-(function, node) shares of the node rows: c (memory = mem_f * c), CPU
//   rpart [F][2][NP] f64 the same memory / c shares at the repaired certificate point
//   bpart [F+JB][NBS] f64 per-block scalars of the small variables
//   ctrl  Ctrl          step sizes, primal weight, restart state, status
// Static (shared by all slots): rows [R] (RowInfo), frow [F+1], D [N][NP] f32, cpr [F][NP] f32,
// gamma [n_int], rho / lo / hi / rownorm [n_dual], cost_int [n_int].
#pragma once
#include <cstdint>

// Build-time variants (A/B-measured on the MI355X):
//   NEP_NT          1: the routing-state streams (x, anchor) use non-temporal loads/stores, so the
//                      once-per-iteration stream does not evict the delay matrix D from the XCD's L2
//   NEP_SPARSE_ANCHOR 1: anchor rows with <= kAnchorK nonzeros are kept as (j, value) pairs (exact
//                      fp32 values: the same anchor, fewer bytes).  0: always dense.
// (An fp16 anchor was measured in round 2 and rejected: certified node LPs fell from 374/384 to
// 70/384 — its rounding re-enters every restart cycle, so the iterates stall above 1e-6.)
#ifndef NEP_NT
#define NEP_NT 1
#endif
#ifndef NEP_SPARSE_ANCHOR
#define NEP_SPARSE_ANCHOR 1
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define NEP_HD __host__ __device__
#else
#define NEP_HD
#endif

namespace nep {

// Step 2, reduced disruption block: the interval of T = sum c - sum old on which the rows D3a/D3b/D4
// (constraints_step2.py:19-55) admit allocated / deallocated within their box, and their LP optimum on it.
//   create (sigma4 = +1):  a <= -T, d <= T, a + d >= -T, a, d <= 0   =>  d = 0, a = -T:  T in [max(0, -ua), -la],
//                          feasible only if ld <= 0 <= ud; cost (w - 1) a = -(w - 1) T
//   delete (sigma4 = -1):  a <= -T, d <= T, a + d >= T,  a, d <= 0   =>  a = 0, d = T:   T in [ld, min(0, ud)],
//                          feasible only if la <= 0 <= ua; cost (w + 1) d = (w + 1) T
// An empty interval (lo > hi) means the box is infeasible.
NEP_HD inline void dred_interval(double sigma4, double la, double ua, double ld, double ud, double &tlo, double &thi) {
  if (sigma4 > 0) {
    const bool ok = ld <= 0.0 && ud >= 0.0;
    tlo = ok ? (-ua > 0.0 ? -ua : 0.0) : 1.0;
    thi = ok ? -la : 0.0;
  } else {
    const bool ok = la <= 0.0 && ua >= 0.0;
    tlo = ok ? ld : 1.0;
    thi = ok ? (ud < 0.0 ? ud : 0.0) : 0.0;
  }
}

// The Halpern anchor is always a point on the routing simplexes (it is set right after a plain
// PDHG step, or from the initial projection), so its rows are sparse: a row keeps up to kAnchorK
// (destination, value) pairs, 8 B each, instead of NP floats.
#ifndef NEP_ANCHOR_K
#define NEP_ANCHOR_K 16
#endif
constexpr int kAnchorK = NEP_ANCHOR_K;   // (build flag for A/B)
constexpr int kAnchorDense = kAnchorK + 1;
struct AnchorEnt {
  int32_t j;
  float v;
};

constexpr int kWave = 64;
constexpr int64_t kOmegaTrained = 1024;  // warm_omega_cap applies when the parent lineage iterated this much
constexpr double kPolishRes = 1e-3;        // polishing entry: primal residual at most this
constexpr int64_t kPolishBudget = 512;     // polishing iterations before the LP goes back to its own objective
constexpr int kNodeWaves = 16;           // waves per node-pass workgroup (each sums F/16 functions)
constexpr int kNodeThreads = kWave * kNodeWaves;
constexpr int kNodeJ = 16;               // nodes per node-pass workgroup

// one routing row (32 B, one scalar load): pooled-row weight m (1 for a single source), workload
// w = W[f, src], objective weight wobj (cost of x[r, j] = wobj * D[src, j]), score-row weight wsc
// (step 2), source node (-1 = the pooled zero-workload sources of f), function f
struct RowInfo {
  float m, w, wobj, wsc;
  int32_t src, f, pad0, pad1;
};

// per-function scalar partials (TS_LAGR_REP: the routing rows' Lagrangian terms at the repaired
// column prices, DESIGN.md §4 "Dual repair")
enum { TS_SCORE = 0, TS_POBJ, TS_LAGR, TS_MOVE, TS_DIST, TS_EMPTY, TS_LAGR_REP, TS_LAGR0, NTS };
// per-block scalar partials of the small variables
enum {
  BS_SUMC_NEW = 0,   // sum over (f,j) of c'            (step-2 rows D3/D4)
  BS_SCORE_N,        // score-row n part of the new n   (step-2 MU/MDU)
  BS_LAGR,           // Lagrangian: small vars + row terms
  BS_POBJ,           // objective of the small vars
  BS_RES,            // max normalised primal violation
  BS_MOVE_Z, BS_MOVE_Y, BS_DIST_Z, BS_DIST_Y,
  BS_SUMC_REP,       // certificate: sum over (f,j) of the repaired c (step-2 rows D3/D4)
  BS_SCORE_N_REP,    // certificate: score-row n part of the repaired n
  BS_LAGR_D,         // step 2: the disruption block's share of the Lagrangian (c, moved, a, d; D1-D4)
  BS_LAGR_REP,       // certificate: the small variables' / node rows' Lagrangian terms at the repaired duals
  BS_TLO, BS_THI,    // step 2: sum over (f,j) of the node box of c (the range of sum c)
  BS_LAGR0,          // certificate: the Lagrangian with the objective off (the infeasibility test)
  BS_LK0,            // step 2: the disruption block kept exact, one sum per price lambda_k of sum c
  BS_LKR0 = BS_LK0 + 6,   //   (kNLam candidates; DESIGN.md §4 "Disruption block"), and the same at the
  NBS = BS_LKR0 + 6       //   repaired column prices (DESIGN.md §4 "Dual repair")
};
constexpr int kNLam = 6;
// BS_POBJ / BS_RES carry, on certificate iterations, the objective of the REPAIRED small variables and
// the max violation of the rows at the repaired point (DESIGN.md §4 "Certificate").

struct Ctrl {
  double eta, omega, tau, sigma;
  double last_restart_fpr, prev_fpr;
  double pobj, lagr, best_lagr, pres, gap;
  double omega_lo, omega_hi;
  int64_t k, k_since_restart, ks_base;   // ks_base: Halpern counter at the block's first iteration
  int64_t max_iters;                     // this LP's iteration limit (nep_lp_opts of its submit)
  int64_t k_lineage;                     // iterations along the warm-start lineage (parent's + own): the
                                         // primal weight counts as adapted (warm cap) from kOmegaTrained on
  int32_t status, active, restart_pending;
  int32_t exact;                         // 1: the node box fixes the objective (see scalar_pass)
  // primal feasibility polishing: once the gap to the best Lagrangian bound is closed
  // and only the primal residual is left, the LP iterates on its feasibility problem (objective 0,
  // duals restarted from 0) from the current point; polish_bound keeps that best bound
  int32_t polish, polish_pending;       // pending: 1 = enter (duals saved, from 0), 2 = leave (duals restored)
  double polish_bound;
  int64_t polish_k0, polish_next;        // iteration polishing started; earliest iteration to start (-1: never)
  double bound_res;                      // > 0: stop with NEP_LP_BOUND once the bound converged (nep_lp_opts)
  int32_t infeas_hits, pad_;             // consecutive certificate checks whose Farkas test held
};

// row-family offsets inside y / kz / rho / lo / hi
struct DualLayout {
  int o1, o2, o3, o5, o6, o7, oD1, oD2, oD3a, oD3b, oD4, oS;
  int oQ;                                // facility relaxation: c[f, j] <= n[j] rows (F*N); else -1
  int n_dual;
};
// small-primal offsets inside zi
struct IntLayout {
  int oc, omf, omt, oa, od, on;
  int n_int;
};

struct DeviceView {
  // sizes
  int N, NP, F, R, JB, CPL;
  int has_n, step2, variant;
  int fac;                               // NEP_RELAX_FACILITY model (nep_fac.hip): x <= c, c <= n, no big-M pairs
  double M, eps, sigma4, cost_n, score_n_coef, w_dis;
  // step 2 with the disruption block reduced (DESIGN.md §4 "Step-2 reduced disruption block"): moved_from /
  // moved_to / allocated / deallocated are not iterated — their LP optimum is a function of c (integral moved
  // bounds: a linear cost per (f, j); allocated / deallocated: one linear cost sT per unit of T = sum c - sum
  // old on an interval of T) — rows D1/D2/D3a/D3b are idle and D4's dual prices the row sum c in [L, U]
  int dred;
  double sT, sum_old;
  DualLayout dl;
  IntLayout il;
  // static
  const RowInfo *rows;
  const int32_t *frow;
  const float *D, *cpr;
  const double *gam, *rho, *lo, *hi, *rownorm, *cost_int, *mem_f;
  const double *capn;                    // [2][N] node memory, node cores (C3 / C5 capacities)
  // per slot (base pointers; slot stride below)
  float *x;
  float *xa;
  int32_t *acnt;                         // [R] anchor nonzeros per row (kAnchorDense: dense in xa)
  AnchorEnt *aent;                       // [R][kAnchorK] sparse anchor rows
  float *theta;                          // [R] last simplex threshold of each routing row (a start hint)
  uint8_t *mask;
  double *zi, *zia, *lb, *ub;
  double *zr;                            // [n_int] the certificate's repaired small variables (last check)
  double *ybak;                          // [n_dual] the duals kept while an LP polishes (Ctrl::polish)
  double *y, *ya, *kz, *kza;             // duals, anchor, activity K z of the iterate and of the anchor
  float *kty;
  double *tpart, *bpart, *npart;
  double *rpart;                         // [F][2][NP] certificate: repaired c shares of the node rows (mem, c)
  Ctrl *ctrl;
  // facility relaxation (fac): the duals of x[r, j] - c[f, j] <= 0, one per routing entry ([R][NP] f32 like x),
  // their Halpern anchor, and per (f, j) their sum over the rows of f (c's reduced cost, next iteration)
  float *lam, *lama, *lsum;
  const float *rho_l;                    // [F][NP] row scale of those rows (the same for every row of f at j)
  int64_t slsum;
  int64_t sx, smask, sint, sdual, skty, stpart, sbpart, snpart, srpart;   // per-slot strides (elements)
  // check/solve parameters.  tol / cutoff / gap tol live in device memory (prm[0..2], written by every
  // nep_lp_submit) because the iteration blocks are replayed from captured HIP graphs: a value
  // passed by value would stay frozen at capture time.
  const double *prm;
  double warm_omega_floor;               // warm starts: primal weight kept >= this x the parent's (0: off)
  double warm_omega_cap;                 // warm starts: primal weight kept <= this x the parent's (0: off)
  double warm_omega_ref;                 // > 0: the floor / cap multiply this instead of the parent's weight
  int64_t polish_after;                  // submit option: polishing may start after this many iterations (-1: never)
  double polish_res;                     // polishing starts only with the primal residual <= this (NEP_POLISH, kPolishRes)
  int64_t polish_budget;                 // polishing iterations before going back to the LP (NEP_POLISH, kPolishBudget)
  // restart rule on the fixed-point residual (sufficient / necessary / artificial, PDLP's 0.2 / 0.8 /
  // 0.36; necessary 0.9 here, measured) and the primal-weight smoothing (0.5); NEP_RESTART /
  // NEP_OMEGA_SMOOTH override them
  double rs_suff, rs_nec, rs_art, omega_smooth;
  int64_t max_iters;
  double bound_res;                      // submit option copied into each new slot's Ctrl (init_slot)
};

// device-to-device segments copied by one launch (nep_aux.hip copy_segments; byte counts multiples of 4)
struct SlotCopy {
  static constexpr int kMax = 12;
  const char *src[kMax];
  char *dst[kMax];
  int64_t bytes[kMax];
  int n;
};
// several slot-state copies in one launch (nep_lp_copy_states): per segment the array base and the slot stride in
// bytes, per pair the source and destination slot; no pair reads or writes a slot another pair of the launch writes
struct SlotCopyN {
  static constexpr int kSeg = 12, kPairs = 32;
  char *base[kSeg];
  int64_t stride[kSeg];
  int32_t src[kPairs], dst[kPairs];
  int nseg, npairs;
};

}  // namespace nep
