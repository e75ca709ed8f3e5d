// nep_aux.hip — gfx950 kernels around the LP solve: what the branch-and-bound and the REST
// response need from a finished node LP, computed where the LP state lives (HBM) so only small
// results cross PCIe.
//
//   node_flows     flow[f, j] = sum_i x[i, f, j] of a slot (the B&B's branching / rounding input;
//                  replaces copying the R x N routing rows to the host)
//   compact_*      the wire format of neptune/utils/output.py:23-39: routing entries x > 0.001 with
//                  np.round(x, 3), allocation entries c > 0.001, as compacted (row, j, value) lists
//   score_check_*  the reference's offline scorers and feasibility checkers
//                  (efttc/utils/objectives.py:23-98, efttc/utils/constraints_step1.py:5-133) on a
//                  slot's solution
// All reductions run in a fixed order (deterministic); no atomics.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>

#include "nep_internal.h"

namespace nep {

// ---------------------------------------------------------------------------------------------
// flows: one workgroup per (function f, slot b); thread = destination j, loop over f's rows
// (coalesced across j).  fp64 accumulation of the pooled-row weights m_r.
// ---------------------------------------------------------------------------------------------
// wout (optional): the same sum over the rows of workload-carrying sources only (the pooled
// zero-workload row excluded: its mass is free to go anywhere)
__global__ __launch_bounds__(256) void node_flows(DeviceView v, const int32_t *__restrict__ slots,
                                                  float *__restrict__ out, float *__restrict__ wout) {
  const int f = blockIdx.x, b = blockIdx.y;
  const int slot = slots[b];
  const float *x = v.x + slot * v.sx;
  const int r0 = v.frow[f], r1 = v.frow[f + 1];
  for (int j = threadIdx.x; j < v.N; j += blockDim.x) {
    double s = 0.0, sw = 0.0;
    for (int r = r0; r < r1; ++r) {
      const double t = (double)v.rows[r].m * (double)x[(int64_t)r * v.NP + j];
      s += t;
      if (v.rows[r].src >= 0) sw += t;
    }
    out[((int64_t)b * v.F + f) * v.N + j] = (float)s;
    if (wout) wout[((int64_t)b * v.F + f) * v.N + j] = (float)sw;
  }
}

// ---------------------------------------------------------------------------------------------
// compaction (deterministic, row order then j order): count per row -> one-workgroup exclusive
// scan -> write.  `vals` is a [rows][ld] matrix (fp32 routing rows, or the fp64 c block viewed
// as F rows of N).
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void compact_count(const T *__restrict__ vals, int rows, int cols, int64_t ld,
                                                     double thr, int32_t *__restrict__ cnt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  int c = 0;
  for (int j = lane; j < cols; j += 64) c += (double)vals[(int64_t)r * ld + j] > thr;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if (lane == 0) cnt[r] = c;
}

// exclusive scan of cnt[0..n) into off[0..n]; one workgroup of 1024 threads, chunked
__global__ __launch_bounds__(1024) void compact_scan(const int32_t *__restrict__ cnt, int n, int32_t *__restrict__ off) {
  __shared__ int32_t part[1024];
  __shared__ int32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const int32_t v = i < n ? cnt[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan
      const int32_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n) off[i] = carry + part[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) off[n] = carry;
}

// write: one wave per row; entries in j order via ballot prefix counts
template <typename T>
__global__ __launch_bounds__(256) void compact_write(const T *__restrict__ vals, int rows, int cols, int64_t ld,
                                                     double thr, int round3, const int32_t *__restrict__ off,
                                                     int32_t *__restrict__ out_row, int32_t *__restrict__ out_col,
                                                     double *__restrict__ out_val) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wave;
  if (r >= rows) return;
  int pos = off[r];
  for (int j0 = 0; j0 < cols; j0 += 64) {
    const int j = j0 + lane;
    const double a = j < cols ? (double)vals[(int64_t)r * ld + j] : 0.0;
    const bool keep = j < cols && a > thr;
    const uint64_t m = __ballot(keep);
    if (keep) {
      const int k = pos + __popcll(m & ((1ull << lane) - 1ull));
      out_row[k] = r;
      out_col[k] = j;
      out_val[k] = round3 ? rint(a * 1000.0) / 1000.0 : a;   // np.round(x, 3) (round half to even)
    }
    pos += __popcll(m);
  }
}

// ---------------------------------------------------------------------------------------------
// scorers / checkers of a slot's solution (efttc/utils/objectives.py, constraints_step1.py).
// Pass 1, one workgroup per (function f, slot): per destination j the flow sum_i x[i,f,j] and the
// CPU share sum_i W[f,i] x[i,f,j] cpr[f,j]; the C1/C2-style c_x check per (f, j); each routing
// row's sum_j x (handle_all_requests, |sum - 1| < 0.1); the network-delay partial of f.
// Pass 2, one thread per node j: CPU, memory, n_c checks and the node partials.
// Pass 3, one workgroup: the slot's totals.
// ---------------------------------------------------------------------------------------------
enum { SC_DELAY = 0, SC_BAD_CX, SC_BAD_HANDLE, SC_BAD_MEM, SC_BAD_CPU, SC_BAD_NC, SC_NUSED, SC_COST, SC_HANDLE_MAXDEV,
       SC_CPU_MAXEXCESS, NSC };

__global__ __launch_bounds__(256) void score_pass_f(DeviceView v, int slot, const double *__restrict__ zi,
                                                    double *__restrict__ cpu_fj, double *__restrict__ fpart) {
  __shared__ double red[4][4];
  const int f = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float *x = v.x + slot * v.sx;
  const int r0 = v.frow[f], r1 = v.frow[f + 1];
  const double M = v.M, eps = v.eps;
  double bad_cx = 0.0, delay = 0.0;
  for (int j = threadIdx.x; j < v.N; j += blockDim.x) {
    double s = 0.0, u = 0.0, dl = 0.0;
    for (int r = r0; r < r1; ++r) {
      const RowInfo ri = v.rows[r];
      const double a = (double)x[(int64_t)r * v.NP + j];
      s += (double)ri.m * a;
      u += (double)ri.w * a;
      if (ri.src >= 0) dl += (double)ri.w * (double)v.D[(int64_t)ri.src * v.NP + j] * a;
    }
    cpu_fj[(int64_t)f * v.NP + j] = u * (double)v.cpr[(int64_t)f * v.NP + j];
    const bool c = zi[v.il.oc + f * v.N + j] != 0.0;   // Python truthiness of c[(f, j)]["val"]
    if (s > (c ? M : 0.0) || s + eps < (c ? 1.0 : 0.0)) bad_cx += 1.0;
    delay += dl;
  }
  // routing-row sums (one wave per row)
  double bad_h = 0.0, maxdev = 0.0;
  for (int r = r0 + wave; r < r1; r += 4) {
    double s = 0.0;
    for (int j = lane; j < v.N; j += 64) s += (double)x[(int64_t)r * v.NP + j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const double dev = fabs(s - 1.0);
    maxdev = fmax(maxdev, dev);
    if (!(dev < 0.1)) bad_h += (double)v.rows[r].m;   // every source the (pooled) row stands for
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    bad_cx += __shfl_xor(bad_cx, o, 64);
    delay += __shfl_xor(delay, o, 64);
  }
  if (lane == 0) {
    red[wave][0] = bad_cx;
    red[wave][1] = delay;
    red[wave][2] = bad_h;   // identical on every lane of the wave (butterfly)
    red[wave][3] = maxdev;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[4] = {0, 0, 0, 0};
    for (int w = 0; w < 4; ++w) {
      t[0] += red[w][0];
      t[1] += red[w][1];
      t[2] += red[w][2];
      t[3] = fmax(t[3], red[w][3]);
    }
    double *p = fpart + (int64_t)f * 4;
    p[0] = t[0]; p[1] = t[1]; p[2] = t[2]; p[3] = t[3];
  }
}

__global__ __launch_bounds__(256) void score_pass_j(DeviceView v, const double *__restrict__ zi,
                                                    const double *__restrict__ cpu_fj,
                                                    const double *__restrict__ node_cost, double budget,
                                                    double *__restrict__ jpart) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= v.N) return;
  const double M = v.M, eps = v.eps;
  double cpu = 0.0, mem = 0.0, sumc = 0.0;
  for (int f = 0; f < v.F; ++f) {
    cpu += cpu_fj[(int64_t)f * v.NP + j];
    const bool c = zi[v.il.oc + f * v.N + j] != 0.0;
    if (c) { mem += v.mem_f[f]; sumc += 1.0; }
  }
  const double cores = v.capn[v.N + j], nmem = v.capn[j];
  double nval = 0.0, nused = 0.0;
  if (v.has_n) {
    nval = zi[v.il.on + j] != 0.0 ? 1.0 : 0.0;
    nused = nval;
  }
  double *p = jpart + (int64_t)j * 6;
  p[0] = cpu > cores + 1e-6 ? 1.0 : 0.0;
  p[1] = mem > nmem ? 1.0 : 0.0;
  p[2] = v.has_n ? ((sumc > nval * M || sumc + eps < nval) ? 1.0 : 0.0) : 0.0;
  p[3] = nused;
  p[4] = v.has_n ? zi[v.il.on + j] * node_cost[j] : 0.0;
  p[5] = fmax(cpu - cores, 0.0);
  (void)budget;
}

__global__ __launch_bounds__(256) void score_final(DeviceView v, const double *__restrict__ fpart,
                                                   const double *__restrict__ jpart, double *__restrict__ out) {
  __shared__ double red[256];
  double acc[NSC];
  for (int k = 0; k < NSC; ++k) acc[k] = 0.0;
  for (int f = threadIdx.x; f < v.F; f += 256) {
    acc[SC_BAD_CX] += fpart[f * 4 + 0];
    acc[SC_DELAY] += fpart[f * 4 + 1];
    acc[SC_BAD_HANDLE] += fpart[f * 4 + 2];
    acc[SC_HANDLE_MAXDEV] = fmax(acc[SC_HANDLE_MAXDEV], fpart[f * 4 + 3]);
  }
  for (int j = threadIdx.x; j < v.N; j += 256) {
    acc[SC_BAD_CPU] += jpart[j * 6 + 0];
    acc[SC_BAD_MEM] += jpart[j * 6 + 1];
    acc[SC_BAD_NC] += jpart[j * 6 + 2];
    acc[SC_NUSED] += jpart[j * 6 + 3];
    acc[SC_COST] += jpart[j * 6 + 4];
    acc[SC_CPU_MAXEXCESS] = fmax(acc[SC_CPU_MAXEXCESS], jpart[j * 6 + 5]);
  }
  for (int k = 0; k < NSC; ++k) {
    const bool mx = k == SC_HANDLE_MAXDEV || k == SC_CPU_MAXEXCESS;
    red[threadIdx.x] = acc[k];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (threadIdx.x < s) red[threadIdx.x] = mx ? fmax(red[threadIdx.x], red[threadIdx.x + s]) : red[threadIdx.x] + red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = red[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// one slot's warm-start state copied to another (nep_lp_copy_state): every segment in one launch instead
// of one hipMemcpyAsync each (8-10 API calls, ~25 us of host time per copy at 64x32).  Segment k (blockIdx.y)
// is bytes[k] bytes, a multiple of 4; 16-byte words where both ends are 16-byte aligned.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void copy_segments(SlotCopy c) {
  const int k = blockIdx.y;
  if (k >= c.n) return;
  const char *src = c.src[k];
  char *dst = c.dst[k];
  const int64_t bytes = c.bytes[k];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t n16 = bytes >> 4;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (int64_t i = t0; i < n16; i += stride) d4[i] = s4[i];
    const int64_t tail = (bytes - (n16 << 4)) >> 2;   // (< 4 words)
    if (t0 < tail) reinterpret_cast<uint32_t *>(dst + (n16 << 4))[t0] = reinterpret_cast<const uint32_t *>(src + (n16 << 4))[t0];
  } else {
    const int64_t n4 = bytes >> 2;
    const uint32_t *s1 = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d1 = reinterpret_cast<uint32_t *>(dst);
    for (int64_t i = t0; i < n4; i += stride) d1[i] = s1[i];
  }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
hipError_t launch_node_flows(const DeviceView &v, const int32_t *slots, int n, float *out, float *wout,
                             hipStream_t s) {
  hipLaunchKernelGGL(node_flows, dim3(v.F, n), dim3(256), 0, s, v, slots, out, wout);
  return hipGetLastError();
}

hipError_t launch_compact_f32(const float *vals, int rows, int cols, int64_t ld, double thr, int round3,
                              int32_t *cnt, int32_t *off, int32_t *orow, int32_t *ocol, double *oval, bool count_only,
                              hipStream_t s) {
  const dim3 g((rows + 3) / 4), b(256);
  if (count_only) {
    hipLaunchKernelGGL(compact_count<float>, g, b, 0, s, vals, rows, cols, ld, thr, cnt);
    hipLaunchKernelGGL(compact_scan, dim3(1), dim3(1024), 0, s, cnt, rows, off);
  } else {
    hipLaunchKernelGGL(compact_write<float>, g, b, 0, s, vals, rows, cols, ld, thr, round3, off, orow, ocol, oval);
  }
  return hipGetLastError();
}

hipError_t launch_compact_f64(const double *vals, int rows, int cols, int64_t ld, double thr, int round3,
                              int32_t *cnt, int32_t *off, int32_t *orow, int32_t *ocol, double *oval, bool count_only,
                              hipStream_t s) {
  const dim3 g((rows + 3) / 4), b(256);
  if (count_only) {
    hipLaunchKernelGGL(compact_count<double>, g, b, 0, s, vals, rows, cols, ld, thr, cnt);
    hipLaunchKernelGGL(compact_scan, dim3(1), dim3(1024), 0, s, cnt, rows, off);
  } else {
    hipLaunchKernelGGL(compact_write<double>, g, b, 0, s, vals, rows, cols, ld, thr, round3, off, orow, ocol, oval);
  }
  return hipGetLastError();
}

// nep_lp_get_solutions: every requested slot's integer vector — the certificate's repaired point for a certified
// slot (status 0), else the iterate — gathered into one buffer, so the host reads n slots with one copy and one
// wait (round 6: it issued 2n copies and two waits, ~10 % of the 64x32 B&B's host time per finished block)
__global__ void gather_solutions(DeviceView v, const int32_t *__restrict__ slots, int ni, double *__restrict__ out) {
  const int b = blockIdx.y;
  const int s = slots[b];
  const double *z = (v.ctrl[s].status == 0 ? v.zr : v.zi) + (int64_t)s * v.sint;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < ni; k += gridDim.x * blockDim.x) out[(int64_t)b * ni + k] = z[k];
}

hipError_t launch_gather_solutions(const DeviceView &v, const int32_t *slots, int n, int ni, double *out,
                                   hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int blocks = std::max(1, std::min(64, (ni + 255) / 256));
  hipLaunchKernelGGL(gather_solutions, dim3(blocks, n), dim3(256), 0, s, v, slots, ni, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void copy_slots(SlotCopyN c) {
  const int k = blockIdx.y, q = blockIdx.z;
  if (k >= c.nseg || q >= c.npairs) return;
  const int64_t bytes = c.stride[k];
  const char *src = c.base[k] + (int64_t)c.src[q] * bytes;
  char *dst = c.base[k] + (int64_t)c.dst[q] * bytes;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    const int64_t n16 = bytes >> 4;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (int64_t i = t0; i < n16; i += stride) d4[i] = s4[i];
    const int64_t tail = (bytes - (n16 << 4)) >> 2;   // (< 4 words)
    if (t0 < tail) reinterpret_cast<uint32_t *>(dst + (n16 << 4))[t0] = reinterpret_cast<const uint32_t *>(src + (n16 << 4))[t0];
  } else {
    const int64_t n4 = bytes >> 2;
    const uint32_t *s1 = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d1 = reinterpret_cast<uint32_t *>(dst);
    for (int64_t i = t0; i < n4; i += stride) d1[i] = s1[i];
  }
}

hipError_t launch_copy_slots(const SlotCopyN &c, hipStream_t s) {
  if (c.nseg <= 0 || c.npairs <= 0) return hipSuccess;
  int64_t most = 0;
  for (int k = 0; k < c.nseg; ++k) most = std::max(most, c.stride[k]);
  // (the pairs share the chip: fewer blocks per segment the more pairs a launch carries)
  const int64_t cap = std::max<int64_t>(16, 1024 / c.npairs);
  const int64_t blocks = std::min<int64_t>(cap, std::max<int64_t>(1, (most / 16 + 255) / 256));
  hipLaunchKernelGGL(copy_slots, dim3((unsigned)blocks, c.nseg, c.npairs), dim3(256), 0, s, c);
  return hipGetLastError();
}

hipError_t launch_copy_segments(const SlotCopy &c, hipStream_t s) {
  if (c.n <= 0) return hipSuccess;
  int64_t most = 0;
  for (int k = 0; k < c.n; ++k) most = std::max(most, c.bytes[k]);
  const int64_t blocks = std::min<int64_t>(1024, std::max<int64_t>(1, (most / 16 + 255) / 256));
  hipLaunchKernelGGL(copy_segments, dim3((unsigned)blocks, c.n), dim3(256), 0, s, c);
  return hipGetLastError();
}

hipError_t launch_score_check(const DeviceView &v, int slot, const double *zi, double *cpu_fj, double *fpart,
                              double *jpart, const double *node_cost, double budget, double *out, hipStream_t s) {
  hipLaunchKernelGGL(score_pass_f, dim3(v.F), dim3(256), 0, s, v, slot, zi, cpu_fj, fpart);
  hipLaunchKernelGGL(score_pass_j, dim3((v.N + 255) / 256), dim3(256), 0, s, v, zi, cpu_fj, node_cost, budget, jpart);
  hipLaunchKernelGGL(score_final, dim3(1), dim3(256), 0, s, v, fpart, jpart, out);
  return hipGetLastError();
}

}  // namespace nep
