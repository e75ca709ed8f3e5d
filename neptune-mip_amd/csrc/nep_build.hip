// nep_build.hip — gfx950 kernels of the model build: the step size eta = 0.95 / ||K̃||_2 by power iteration on
// K̃ᵀK̃ (K̃ = diag(rho) K diag(1, gam): the routing columns keep scale 1) over the model's structured rows, in fp64,
// on the device (nep_model_create; DESIGN.md §6 "Device build").  The same operator as the host power iteration
// nep_debug_build keeps (nep_host.cpp power_host), from the same start vector: 60 passes over the R x N routing
// entries took 1.5-6 s of host time per 512x256 model (two thirds of its build), ~10 ms here.
//
//   pi_fwd_rows   per function f (one workgroup): column sums S[f, j] of its rows into the C1/C2 rows, the
//                 W-weighted CPU shares U[f, j] (-> C5) and the score-row share (step 2)
//   pi_fwd_nodes  C5 rows: sum over f of U[f, j]; the score row: sum of the function shares (fixed order)
//   pi_fwd_coo    the small-variable part of K (CSR of the scaling matrix) and the row scales: w = rho² (K z)
//   pi_bwd_rows   K̃ᵀ w on the routing entries (facility relaxation: its x <= c rows, scale rhoL, folded in)
//   pi_bwd_cols   K̃ᵀ w on the small variables (CSC), times gam
//   dot2 / dot_finish / scale2   fixed-order reductions (deterministic) and the normalisation
#include <hip/hip_runtime.h>
#include <cmath>

#include "nep_internal.h"

namespace nep {

constexpr int kPiThreads = 256;

__device__ __forceinline__ double block_sum(double v, double *sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += sh[k];
  __syncthreads();
  return t;   // (valid in thread 0)
}

template <bool FAC>
__global__ __launch_bounds__(kPiThreads) void pi_fwd_rows(DeviceView v, const double *__restrict__ zx,
                                                          double *__restrict__ y, double *__restrict__ upart,
                                                          double *__restrict__ spart) {
  __shared__ double sh[kPiThreads / 64];
  const int f = blockIdx.x, N = v.N, NP = v.NP;
  const int r0 = v.frow[f], r1 = v.frow[f + 1];
  double sc = 0.0;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    double S = 0.0, U = 0.0;
    for (int r = r0; r < r1; ++r) {
      const RowInfo ri = v.rows[r];
      const double z = zx[(int64_t)r * N + j];
      S += (double)ri.m * z;
      U += (double)ri.w * z;
      if (ri.src >= 0 && ri.wsc != 0.f) sc += (double)ri.wsc * (double)v.D[(int64_t)ri.src * NP + j] * z;
    }
    if (!FAC) {
      y[v.dl.o1 + f * N + j] = S;
      y[v.dl.o2 + f * N + j] = S;
    }
    upart[(int64_t)f * N + j] = U * (double)v.cpr[(int64_t)f * NP + j];
  }
  const double t = block_sum(sc, sh);
  if (threadIdx.x == 0) spart[f] = t;
}

__global__ __launch_bounds__(kPiThreads) void pi_fwd_nodes(DeviceView v, const double *__restrict__ upart,
                                                           const double *__restrict__ spart, double *__restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < v.N) {
    double U = 0.0;
    for (int f = 0; f < v.F; ++f) U += upart[(int64_t)f * v.N + j];
    y[v.dl.o5 + j] = U;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && v.step2) {
    double s = 0.0;
    for (int f = 0; f < v.F; ++f) s += spart[f];
    y[v.dl.oS] = s;
  }
}

__global__ __launch_bounds__(kPiThreads) void pi_fwd_coo(DeviceView v, int n_dual, const int32_t *__restrict__ rp,
                                                         const int32_t *__restrict__ ci, const double *__restrict__ cv,
                                                         const double *__restrict__ zs, double *__restrict__ y) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_dual) return;
  double acc = y[k];
  for (int e = rp[k]; e < rp[k + 1]; ++e) acc += cv[e] * v.gam[ci[e]] * zs[ci[e]];
  const double rr = v.rho[k];
  y[k] = rr * rr * acc;   // rho (K̃ z), ready for K̃ᵀ
}

template <bool FAC>
__global__ __launch_bounds__(kPiThreads) void pi_bwd_rows(DeviceView v, const double *__restrict__ w,
                                                          const double *__restrict__ zx, const double *__restrict__ zs,
                                                          double *__restrict__ gx, double *__restrict__ gfac) {
  const int f = blockIdx.x, N = v.N, NP = v.NP;
  const int r0 = v.frow[f], r1 = v.frow[f + 1];
  const double wS = v.step2 ? w[v.dl.oS] : 0.0;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const double w5 = w[v.dl.o5 + j] * (double)v.cpr[(int64_t)f * NP + j];
    const double w12 = FAC ? 0.0 : w[v.dl.o1 + f * N + j] + w[v.dl.o2 + f * N + j];
    double rl = 0.0, gc = 0.0, zc = 0.0, tsum = 0.0;
    if (FAC) {
      rl = (double)v.rho_l[(int64_t)f * NP + j];
      gc = v.gam[v.il.oc + f * N + j];
      zc = zs[v.il.oc + f * N + j];
    }
    for (int r = r0; r < r1; ++r) {
      const RowInfo ri = v.rows[r];
      double g = (double)ri.w * w5 + (double)ri.m * w12;
      if (ri.src >= 0 && ri.wsc != 0.f) g += (double)ri.wsc * (double)v.D[(int64_t)ri.src * NP + j] * wS;
      if (FAC) {   // the x <= c rows: t = rhoL (x - gam_c z_c); x gets rhoL t, z_c gets -rhoL t
        const double t = rl * (zx[(int64_t)r * N + j] - gc * zc);
        g += rl * t;
        tsum += rl * t;
      }
      gx[(int64_t)r * N + j] = g;
    }
    if (FAC) gfac[f * N + j] = tsum;
  }
}

__global__ __launch_bounds__(kPiThreads) void pi_bwd_cols(DeviceView v, const int32_t *__restrict__ cp,
                                                          const int32_t *__restrict__ ri, const double *__restrict__ rv,
                                                          const double *__restrict__ w, const double *__restrict__ gfac,
                                                          double *__restrict__ gs) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= v.il.n_int) return;
  double acc = 0.0;
  for (int e = cp[c]; e < cp[c + 1]; ++e) acc += rv[e] * w[ri[e]];
  if (v.fac && c >= v.il.oc && c < v.il.oc + v.F * v.N) acc -= gfac[c - v.il.oc];
  gs[c] = v.gam[c] * acc;
}

// partial sums of a1·b1 (n1 entries) + a2·b2 (n2 entries), one per block, fixed order
__global__ __launch_bounds__(kPiThreads) void dot2(const double *__restrict__ a1, const double *__restrict__ b1,
                                                   int64_t n1, const double *__restrict__ a2,
                                                   const double *__restrict__ b2, int64_t n2,
                                                   double *__restrict__ part) {
  __shared__ double sh[kPiThreads / 64];
  double s = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2; i += stride)
    s += i < n1 ? a1[i] * b1[i] : a2[i - n1] * b2[i - n1];
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void dot_finish(const double *__restrict__ part, int n, double *__restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int k = 0; k < n; ++k) s += part[k];
    *out = s;
  }
}

// a1 /= sqrt(*sq), a2 /= sqrt(*sq)
__global__ __launch_bounds__(kPiThreads) void scale2(double *__restrict__ a1, int64_t n1, double *__restrict__ a2,
                                                     int64_t n2, const double *__restrict__ sq) {
  const double s = 1.0 / sqrt(*sq);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n1 + n2; i += stride) {
    if (i < n1) a1[i] *= s;
    else a2[i - n1] *= s;
  }
}

// One power-iteration run: zx [R][N] and zs [n_int] hold the start vector; gx / gs are scratch of the same sizes,
// y [n_dual], upart [F][N], spart [F], gfac [F][N], part [nblk], out [iters + 1] (out[1 + it] = lambda of pass it).
// CSR (rp, ci, cv) / CSC (cp, ri, rv) of the small-variable part of the scaling matrix.
hipError_t launch_power_iteration(const DeviceView &v, int iters, double *zx, double *zs, double *gx, double *gs,
                                  double *y, double *upart, double *spart, double *gfac, double *part, int nblk,
                                  double *out, const int32_t *rp, const int32_t *ci, const double *cv,
                                  const int32_t *cp, const int32_t *ri, const double *rv, hipStream_t s) {
  const int64_t nx = (int64_t)v.R * v.N, nz = v.il.n_int;
  const int nd = v.dl.n_dual;
  for (int it = 0; it < iters; ++it) {
    dot2<<<nblk, kPiThreads, 0, s>>>(zx, zx, nx, zs, zs, nz, part);
    dot_finish<<<1, 64, 0, s>>>(part, nblk, out);
    scale2<<<nblk, kPiThreads, 0, s>>>(zx, nx, zs, nz, out);
    hipError_t e = hipMemsetAsync(y, 0, sizeof(double) * nd, s);
    if (e != hipSuccess) return e;
    if (v.fac) pi_fwd_rows<true><<<v.F, kPiThreads, 0, s>>>(v, zx, y, upart, spart);
    else pi_fwd_rows<false><<<v.F, kPiThreads, 0, s>>>(v, zx, y, upart, spart);
    pi_fwd_nodes<<<(v.N + kPiThreads - 1) / kPiThreads, kPiThreads, 0, s>>>(v, upart, spart, y);
    pi_fwd_coo<<<(nd + kPiThreads - 1) / kPiThreads, kPiThreads, 0, s>>>(v, nd, rp, ci, cv, zs, y);
    if (v.fac) pi_bwd_rows<true><<<v.F, kPiThreads, 0, s>>>(v, y, zx, zs, gx, gfac);
    else pi_bwd_rows<false><<<v.F, kPiThreads, 0, s>>>(v, y, zx, zs, gx, gfac);
    pi_bwd_cols<<<(int)((nz + kPiThreads - 1) / kPiThreads), kPiThreads, 0, s>>>(v, cp, ri, rv, y, gfac, gs);
    dot2<<<nblk, kPiThreads, 0, s>>>(zx, gx, nx, zs, gs, nz, part);
    dot_finish<<<1, 64, 0, s>>>(part, nblk, out + 1 + it);
    double *t = zx; zx = gx; gx = t;
    t = zs; zs = gs; gs = t;
  }
  return hipGetLastError();
}

}  // namespace nep
