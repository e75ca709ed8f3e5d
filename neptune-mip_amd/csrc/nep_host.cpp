// nep_host.cpp — host runtime of the NEPTUNE LP engine: model build (exact zero-workload
// aggregation, coefficients, diagonal scaling, step size), per-node presolve, the batched PDHG
// solve loop on one HIP stream (batch and streaming forms), solution export, and the extern "C"
// ABI of include/neptune_lp.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <random>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_lp.h"
#include "nep_internal.h"

namespace nep {
hipError_t launch_x_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                         bool plain, int it, hipStream_t s);
hipError_t launch_node_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init, bool first,
                            bool plain, int it, hipStream_t s);
hipError_t launch_scalar_pass(const DeviceView &v, const int32_t *slots, int nslots, bool check, bool init,
                              bool first, bool plain, int it, int block_len, hipStream_t s);
hipError_t launch_node_bounds(const DeviceView &v, const int32_t *slots, int nslots, const double *base_lb,
                              const double *base_ub, const uint8_t *base_mask, const int32_t *off, const int32_t *idx,
                              const double *cl, const double *cu, int max_chg, hipStream_t s);
hipError_t launch_init_slot(const DeviceView &v, const int32_t *slots, const int32_t *exact, int nslots, bool warm,
                            double eta, double omega0, const double *per, hipStream_t s);
hipError_t launch_node_flows(const DeviceView &v, const int32_t *slots, int n, float *out, float *wout,
                             hipStream_t s);
hipError_t launch_compact_f32(const float *vals, int rows, int cols, int64_t ld, double thr, int round3,
                              int32_t *cnt, int32_t *off, int32_t *orow, int32_t *ocol, double *oval, bool count_only,
                              hipStream_t s);
hipError_t launch_compact_f64(const double *vals, int rows, int cols, int64_t ld, double thr, int round3,
                              int32_t *cnt, int32_t *off, int32_t *orow, int32_t *ocol, double *oval, bool count_only,
                              hipStream_t s);
hipError_t launch_copy_segments(const SlotCopy &c, hipStream_t s);
hipError_t launch_copy_slots(const SlotCopyN &c, hipStream_t s);
hipError_t launch_gather_solutions(const DeviceView &v, const int32_t *slots, int n, int ni, double *out,
                                   hipStream_t s);
hipError_t launch_power_iteration(const DeviceView &v, int iters, double *zx, double *zs, double *gx, double *gs,
                                  double *y, double *upart, double *spart, double *gfac, double *part, int nblk,
                                  double *out, const int32_t *rp, const int32_t *ci, const double *cv,
                                  const int32_t *cp, const int32_t *ri, const double *rv, hipStream_t s);
hipError_t launch_score_check(const DeviceView &v, int slot, const double *zi, double *cpu_fj, double *fpart,
                              double *jpart, const double *node_cost, double budget, double *out, hipStream_t s);
}  // namespace nep

using namespace nep;

static thread_local std::string g_err;
static int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}
namespace nep {
int set_error(int code, const char *msg) { return fail(code, msg ? msg : ""); }   // (nep_bnb.cpp's messages)
}
#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) return fail(NEP_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

static const double INF = std::numeric_limits<double>::infinity();
// NEP_HALPERN=0 (A/B build variant): plain restarted PDHG — every iteration w' = T(w), the anchor is
// read only on certificate iterations (restart distances)
#ifndef NEP_HALPERN
#define NEP_HALPERN 1
#endif
static constexpr bool kHalpern = NEP_HALPERN != 0;

namespace {

struct Coo {
  std::vector<int> r, c;
  std::vector<double> v;
  void add(int row, int col, double val) {
    r.push_back(row);
    c.push_back(col);
    v.push_back(val);
  }
};

// scratch of one presolve_node() call, reset after every node (one per thread)
struct PresolveScratch {
  std::vector<int> pos, fdelta, touched, ftouched;
  std::vector<double> dmin, dmax;
  std::vector<uint8_t> rowmark;
  std::vector<uint8_t> allow;   // [F*N] the node's allowed placements (CPU cover and score-row tests)
  // the changes of the nodes this thread presolved in the current batch (capacity kept across batches: a
  // rounding leaf's ~33k changes at 256x128 would otherwise page-fault fresh buffers on every submit)
  std::vector<int32_t> ci;
  std::vector<double> cl, cu;
};

struct Model {
  // NEP_HOST_PROFILE=1: host seconds of nep_lp_submit (presolve / staging + launches) and nep_lp_advance,
  // printed to stderr when the model is destroyed (dev measurement)
  bool prof = false;
  double pr_pre = 0, pr_stage = 0, pr_adv = 0;
  int64_t pr_calls = 0, pr_lps = 0, pr_adv_calls = 0;
  // problem
  int N = 0, F = 0, NP = 0, variant = 0, step = 1, has_n = 0, step2 = 0;
  int fac = 0;                      // NEP_RELAX_FACILITY (include/neptune_lp.h)
  std::vector<double> rhoL;         // fac: row scale of the x[r, j] <= c[f, j] rows, per (f, j)
  std::vector<double> capn;         // [2][N] node memory, node cores
  double alpha = 0.5, M = 1e6, eps = 1e-6, sigma4 = -1, cost_n = 0, score_n_coef = 0, w_dis = 0;
  int dred = 0;                     // step 2: the reduced disruption block (DeviceView::dred)
  Coo Ks;                           // the small-variable part of the matrix the iteration runs on (scaling, power)
  bool power_host = false;          // eta from the host power iteration (nep_debug_build) or the device's
  double sT = 0, sum_old = 0;       // dred: cost per unit of T = sum c - sum old; sum of the old allocation
  int R = 0, JB = 0, CPL = 1, max_batch = 1;
  DualLayout dl{};
  IntLayout il{};
  std::vector<int> row_f, row_src, frow;
  std::vector<float> row_m, row_w, row_wobj, row_wsc;
  std::vector<double> row_wsc_d;    // the score-row weights in fp64 (presolve's proofs; row_wsc is the kernels' fp32)
  std::vector<RowInfo> rows;
  std::vector<double> W;            // [F*N]
  std::vector<double> cprh;         // [F*N] core_per_req (the presolve's CPU cover test)
  std::vector<double> wsum;         // [F] sum_i W[f, i]
  std::vector<double> nat_lb, nat_ub, cost_int;
  std::vector<double> lo, hi, rownorm, rho, gam;
  std::vector<double> mem_f;
  // non-x part of K (COO) and, per function, the total routed flow (= N sources x 1): kept for the
  // per-node row-activity test of presolve()
  std::vector<int> Kr, Kc;
  std::vector<double> Kv, ftot;
  bool x_coef_nonneg = true;   // every x coefficient outside C1/C2 is >= 0 (W, cpr, D >= 0)
  // step 2: the score / delay row's routing coefficients wsc[r] * D[src, j] (presolve: the row's smallest
  // activity over the routing simplexes of a node's allowed destinations)
  bool score_x = false;
  std::vector<double> Dh;            // [N*N] delay matrix (step 2 with score_x only)
  bool x_cost_free = true;     // no routing entry carries objective cost (step 2; W == 0)
  // node presolve as a sparse change of the base box (presolve_setup / presolve_node)
  bool base_ok = false;
  std::vector<double> base_lb, base_ub, base_amin, base_amax;
  std::vector<uint8_t> base_mask;
  std::vector<int> base_cnt, Kcp, Kcr;
  std::vector<double> Kcv;
  std::vector<PresolveScratch> psc;   // one per presolve thread (submit presolves a batch's nodes in parallel)
  double eta = 0, sigma_max = 0, omega0 = 1.0;
  double omega_ref = 0.0;           // nep_lp_set_reference_weight (0: warm-start band relative to the parent)
  // device
  hipStream_t stream = nullptr;
  bool own_stream = false;
  // auxiliary stream: work on slots that are NOT iterating — the initialisation of newly submitted
  // slots, warm-start copies and every read of a finished slot (flows, solution, compaction, scorers)
  // — so none of it queues behind the pipelined block on `stream`; ev_aux orders `stream` after it
  hipStream_t aux = nullptr;
  hipEvent_t ev_aux = nullptr;
  DeviceView v{};
  std::vector<void *> allocs;
  double *d_prm = nullptr;      // {tol, cutoff} of the LPs in flight (DeviceView::prm)
  double prm_host[3] = {0, 0, 0};   // tol, cutoff, gap tol of the LPs in flight
  bool prm_sent = false;            // d_prm holds prm_host (a submit with the same values skips the copy)
  int32_t *d_slots = nullptr;   // the slots currently iterating (mirror of `act`)
  int32_t *h_act = nullptr;     // pinned staging of `act` for the d_slots upload (launch_block only)
  int32_t *d_new = nullptr;     // slots being initialised by nep_lp_submit
  double *d_base_lb = nullptr, *d_base_ub = nullptr;
  uint8_t *d_base_mask = nullptr;
  // a submit's uploads, one copy each: [slots | change offsets | change indices | exact flags] and
  // [change lower bounds | change upper bounds] (capacity: every integer variable of every slot)
  int32_t *d_sub_i = nullptr;
  double *d_sub_d = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  nep_stats stats{};
  // scratch of the auxiliary kernels (nep_aux.hip), allocated on first use
  float *d_flows = nullptr;                  // [max_batch][F][N]
  int32_t *d_cnt = nullptr, *d_off = nullptr;   // [max(R, F) + 1]
  int32_t *d_erow = nullptr, *d_ecol = nullptr;
  double *d_eval = nullptr;
  int64_t ecap = 0;
  double *d_score = nullptr;                 // cpu_fj [F][NP] | fpart [F][4] | jpart [N][6] | out [16]
  double *d_node_cost = nullptr;
  std::vector<double> node_cost;
  double node_budget = 0.0;
  // one block of check_every PDHG iterations as a captured HIP graph, per iterating-slot count
  // (the launch grids depend on it); rebuilt when check_every changes
  std::vector<hipGraphExec_t> block_graph;   // [max_batch + 1], index = slots iterating
  int graph_ce = 0;
  int64_t blocks = 0;
  bool graphs_ok = true;                     // false once capture failed on this stream: eager blocks
  // streaming state
  std::vector<int32_t> act;     // slots currently iterating
  std::vector<uint8_t> busy;    // per slot: iterating
  nep_lp_opts run{};            // options of the LPs in flight
  // pipelined blocks (advance): the block launched last, not yet waited for — the slots it iterates,
  // whether it carries the sampled x-pass events — and the pinned copy of the slots' Ctrl it ends with
  bool inflight = false, inflight_sampled = false;
  int pipe_max_done = INT_MAX;
  std::vector<int32_t> launched;
  Ctrl *h_ctrl = nullptr;
  float *h_flows = nullptr;     // pinned staging of nep_lp_get_flows(_split): [2][max_batch][F*N] + slots
  double *h_sols = nullptr;     // pinned staging of nep_lp_get_solutions: [max_batch][n_int] + the slot list
  double *d_sols = nullptr;     // [max_batch][n_int]: the gathered solutions (gather_solutions)
  // pinned staging of nep_lp_submit's uploads (slots, change offsets / indices / bounds, exact flags): the
  // call returns without waiting for them; two stagings alternate, and a submit waits on the event of the
  // one it rewrites (recorded after that staging's copies, two submits earlier: normally long done)
  int32_t *h_sub_i[2] = {nullptr, nullptr};
  double *h_sub_d[2] = {nullptr, nullptr};
  size_t cap_sub_i[2] = {0, 0}, cap_sub_d[2] = {0, 0};
  hipEvent_t ev_sub[2] = {nullptr, nullptr};
  bool sub_pending[2] = {false, false};
  int sub_k = 0;
  ~Model() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (aux) (void)hipStreamSynchronize(aux);
    if (h_ctrl) (void)hipHostFree(h_ctrl);
    if (h_act) (void)hipHostFree(h_act);
    if (h_flows) (void)hipHostFree(h_flows);
    if (h_sols) (void)hipHostFree(h_sols);
    for (int k = 0; k < 2; ++k) {
      if (h_sub_i[k]) (void)hipHostFree(h_sub_i[k]);
      if (h_sub_d[k]) (void)hipHostFree(h_sub_d[k]);
      if (ev_sub[k]) (void)hipEventDestroy(ev_sub[k]);
    }
    for (void *p : allocs) (void)hipFree(p);
    for (hipGraphExec_t g : block_graph)
      if (g) (void)hipGraphExecDestroy(g);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev_aux) (void)hipEventDestroy(ev_aux);
    if (aux) (void)hipStreamDestroy(aux);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }
};

template <typename T>
int dalloc(Model &m, T **p, size_t n) {
  void *q = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc(&q, n * sizeof(T));
  if (e != hipSuccess) return fail(NEP_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  m.allocs.push_back(q);
  *p = static_cast<T *>(q);
  return NEP_OK;
}
template <typename T>
int upload(Model &m, const T **dst, const std::vector<T> &src) {
  T *p = nullptr;
  int rc = dalloc(m, &p, src.size());
  if (rc) return rc;
  if (!src.empty()) {
    hipError_t e = hipMemcpy(p, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(NEP_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  *dst = p;
  return NEP_OK;
}

// ---------------------------------------------------------------------------------------------
// model build
// ---------------------------------------------------------------------------------------------
int build(Model &m, const nep_model_desc &d, bool host_power = true) {
  const int N = d.n_nodes, F = d.n_functions;
  if (N <= 0 || F <= 0) return fail(NEP_ERR_ARG, "n_nodes and n_functions must be positive");
  if (N > 2048) return fail(NEP_ERR_ARG, "n_nodes > 2048 not supported by this build");
  if (d.variant < 0 || d.variant > 2) return fail(NEP_ERR_ARG, "bad variant");
  if (d.step < 1 || d.step > 3) return fail(NEP_ERR_ARG, "bad step");
  if (!d.delay || !d.workload || !d.core_per_req || !d.function_memory || !d.node_memory || !d.node_cores ||
      !d.node_cost || !d.max_delay)
    return fail(NEP_ERR_ARG, "missing input array");
  if (d.step != NEP_STEP1 && !d.old_allocations) return fail(NEP_ERR_ARG, "step 2 needs old_allocations");
  m.N = N;
  m.F = F;
  m.variant = d.variant;
  m.step = d.step;
  m.step2 = d.step != NEP_STEP1;
  m.has_n = d.variant != NEP_MIN_DELAY;
  if (d.relaxation != NEP_RELAX_REFERENCE && d.relaxation != NEP_RELAX_FACILITY) return fail(NEP_ERR_ARG, "bad relaxation");
  m.fac = d.relaxation == NEP_RELAX_FACILITY;
  if (m.fac && (m.step2 || !m.has_n))
    return fail(NEP_ERR_ARG, "the facility relaxation is a step-1 MinUtilization / MinDelayAndUtilization model");
  m.alpha = d.alpha;
  m.M = d.big_m > 0 ? d.big_m : 1e6;
  m.eps = d.epsilon > 0 ? d.epsilon : 1e-6;
  m.sigma4 = d.step == NEP_STEP2_CREATE ? 1.0 : -1.0;
  m.NP = (N + 3) / 4 * 4;
  const int chunks = m.NP / 4;
  m.CPL = chunks <= 64 ? 1 : chunks <= 128 ? 2 : chunks <= 256 ? 4 : 8;
  m.W.assign(d.workload, d.workload + (size_t)F * N);
  m.cprh.assign(d.core_per_req, d.core_per_req + (size_t)F * N);
  m.wsum.assign(F, 0.0);
  for (int f = 0; f < F; ++f)
    for (int i = 0; i < N; ++i) m.wsum[f] += m.W[(size_t)f * N + i];
  const double *D = d.delay;

  // exact aggregation of zero-workload sources: they enter only the column sums (C1/C2) and their
  // own C4 row, with zero objective / CPU / score coefficients, so one pooled row of weight
  // m_f = #zero sources carries them all (x[i,f,:] = pooled row for every such i).
  for (int f = 0; f < F; ++f) {
    int zeros = 0;
    for (int i = 0; i < N; ++i) {
      const double w = m.W[(size_t)f * N + i];
      if (w != 0.0) {
        m.row_f.push_back(f);
        m.row_src.push_back(i);
        m.row_m.push_back(1.f);
        m.row_w.push_back((float)w);
      } else {
        ++zeros;
      }
    }
    if (zeros > 0) {
      m.row_f.push_back(f);
      m.row_src.push_back(-1);
      m.row_m.push_back((float)zeros);
      m.row_w.push_back(0.f);
    }
  }
  m.R = (int)m.row_f.size();

  // objective / score coefficients (objectives.py:4-52, constraints_step2.py:57-88)
  double sumW = 0.0;
  for (double w : m.W) sumW += w;
  double kobj = 0.0;
  if (!m.step2) {
    if (d.variant == NEP_MIN_DELAY) {
      kobj = 1.0;
    } else if (d.variant == NEP_MIN_DELAY_AND_UTILIZATION && sumW != 0.0) {
      double mwd = 0.0;   // objectives.py:36-43
      for (int f = 0; f < F; ++f)
        for (int i = 0; i < N; ++i) {
          double best = -INF;
          for (int j = 0; j < N; ++j) {
            const double dl = D[(size_t)i * N + j];
            if (dl <= d.max_delay[f]) best = std::max(best, dl);
          }
          if (best == -INF) return fail(NEP_ERR_ARG, "max() of an empty delay set (objectives.py:41)");
          mwd += m.W[(size_t)f * N + i] * best;
        }
      if (mwd == 0.0) return fail(NEP_ERR_ARG, "max_workload_delay == 0: division by zero (objectives.py:50)");
      kobj = (1.0 - d.alpha) / mwd;
    }
    m.cost_n = d.variant == NEP_MIN_UTILIZATION ? 1.0 : d.variant == NEP_MIN_DELAY_AND_UTILIZATION ? d.alpha / N : 0.0;
  }
  double score_rhs = INF;
  std::vector<double> colmaxD(N, -INF);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < N; ++i) colmaxD[i] = std::max(colmaxD[i], D[(size_t)k * N + i]);
  m.row_wobj.resize(m.R);
  m.row_wsc.resize(m.R);
  m.row_wsc_d.assign(m.R, 0.0);
  for (int r = 0; r < m.R; ++r) {
    m.row_wobj[r] = (float)(kobj * m.row_w[r]);
    double wsc = 0.0;
    if (m.step2 && m.row_src[r] >= 0) {
      const int f = m.row_f[r], i = m.row_src[r];
      const double wd = m.W[(size_t)f * N + i];
      if (d.variant == NEP_MIN_DELAY) wsc = wd;
      else if (d.variant == NEP_MIN_DELAY_AND_UTILIZATION)
        wsc = (1.0 - d.alpha) * wd / std::max(d.max_delay[f], colmaxD[i]);
    }
    m.row_wsc[r] = (float)wsc;
    m.row_wsc_d[r] = wsc;
    if (wsc != 0.0) m.score_x = true;
  }
  if (m.score_x) m.Dh.assign(D, D + (size_t)N * N);
  if (m.step2) {
    if (d.variant == NEP_MIN_DELAY) {
      score_rhs = d.soften_step1_sol * d.prev_network_delay;
      m.score_n_coef = 0.0;
    } else {
      score_rhs = d.max_score * d.soften_step1_sol;
      m.score_n_coef = d.variant == NEP_MIN_UTILIZATION ? 1.0 : d.alpha / N;
    }
  }

  // rows of one function are consecutive: frow[f] .. frow[f+1] (one x-pass workgroup each)
  m.frow.assign(F + 1, 0);
  for (int r = 0; r < m.R; ++r) m.frow[m.row_f[r] + 1] += 1;
  for (int f = 0; f < F; ++f) m.frow[f + 1] += m.frow[f];
  m.rows.resize(m.R);
  for (int r = 0; r < m.R; ++r)
    m.rows[r] = RowInfo{m.row_m[r], m.row_w[r], m.row_wobj[r], m.row_wsc[r], m.row_src[r], m.row_f[r], 0, 0};
  m.JB = (N + kNodeJ - 1) / kNodeJ;   // node-pass workgroups per LP

  // integer-variable layout (variables.py order minus x)
  const int FN = F * N;
  IntLayout &il = m.il;
  il.oc = 0;
  if (!m.step2) {
    il.omf = il.omt = il.oa = il.od = -1;
    il.on = m.has_n ? FN : -1;
    il.n_int = FN + (m.has_n ? N : 0);
  } else {
    il.omf = FN;
    il.omt = 2 * FN;
    il.oa = 3 * FN;
    il.od = 3 * FN + 1;
    il.on = m.has_n ? 3 * FN + 2 : -1;
    il.n_int = 3 * FN + 2 + (m.has_n ? N : 0);
  }
  m.nat_lb.assign(il.n_int, 0.0);
  m.nat_ub.assign(il.n_int, 1.0);
  m.cost_int.assign(il.n_int, 0.0);
  if (m.has_n)
    for (int j = 0; j < N; ++j) {
      // C8 (constraints_step1.py:101-103): cost[j] * n[j] <= budget  ->  bound on n
      if (d.node_cost[j] > 0) m.nat_ub[il.on + j] = std::min(1.0, d.node_budget / d.node_cost[j]);
      else if (d.node_budget < 0) m.nat_ub[il.on + j] = -1.0;   // infeasible budget row
      m.cost_int[il.on + j] = m.cost_n;
    }
  double sum_old = 0.0;
  if (m.step2) {
    m.w_dis = (double)FN;   // objectives.py:56  w = np.ma.size(old)
    for (int k = 0; k < FN; ++k) {
      m.cost_int[il.omf + k] = m.w_dis;
      m.cost_int[il.omt + k] = m.w_dis;
      sum_old += d.old_allocations[k];
    }
    m.cost_int[il.oa] = m.w_dis - 1;
    m.cost_int[il.od] = m.w_dis + 1;
    m.nat_lb[il.oa] = m.nat_lb[il.od] = -(double)FN;
    m.nat_ub[il.oa] = m.nat_ub[il.od] = 0.0;
  }

  // dual layout + row bounds
  DualLayout &dl = m.dl;
  int o = 0;
  dl.o1 = dl.o2 = dl.oQ = -1;
  if (!m.fac) { dl.o1 = o; o += FN; dl.o2 = o; o += FN; }
  dl.o3 = o; o += N;
  dl.o5 = o; o += N;
  dl.o6 = dl.o7 = dl.oD1 = dl.oD2 = dl.oD3a = dl.oD3b = dl.oD4 = dl.oS = -1;
  if (m.fac) { dl.oQ = o; o += FN; }   // c[f, j] - n[j] <= 0
  else if (m.has_n) { dl.o6 = o; o += N; dl.o7 = o; o += N; }
  if (m.step2) {
    dl.oD1 = o; o += FN;
    dl.oD2 = o; o += FN;
    dl.oD3a = o++; dl.oD3b = o++; dl.oD4 = o++; dl.oS = o++;
  }
  dl.n_dual = o;
  m.lo.assign(o, -INF);
  m.hi.assign(o, INF);
  for (int k = 0; k < FN && !m.fac; ++k) {
    m.hi[dl.o1 + k] = 0.0;
    m.lo[dl.o2 + k] = -m.eps;
  }
  for (int k = 0; k < FN && m.fac; ++k) m.hi[dl.oQ + k] = 0.0;
  m.capn.resize(2 * (size_t)N);
  for (int j = 0; j < N; ++j) {
    m.capn[j] = d.node_memory[j];
    m.capn[N + j] = d.node_cores[j];
    // (fac: C3 / C5 carry n[j] on the right, mem c - Mem_j n <= 0 and CPU - cores_j n <= 0)
    m.hi[dl.o3 + j] = m.fac ? 0.0 : d.node_memory[j];
    m.hi[dl.o5 + j] = m.fac ? 0.0 : d.node_cores[j];
    if (m.has_n && !m.fac) { m.hi[dl.o6 + j] = 0.0; m.lo[dl.o7 + j] = -m.eps; }
  }
  if (m.step2) {
    for (int k = 0; k < FN; ++k) {
      m.lo[dl.oD1 + k] = -d.old_allocations[k];
      m.lo[dl.oD2 + k] = d.old_allocations[k];
    }
    m.lo[dl.oD3a] = -sum_old;
    m.lo[dl.oD3b] = sum_old;
    m.lo[dl.oD4] = m.sigma4 * sum_old;
    m.hi[dl.oS] = score_rhs;
  }
  // Step 2, reduced disruption block: with integral moved_from / moved_to bounds the LP optimum
  // has mf = max(lb_mf, c - old), mt = max(lb_mt, old - c) — a linear cost in c per (f, j) — and the rows
  // D3a/D3b/D4 force (create) d = 0, a = -T or (delete) a = 0, d = T for T = sum c - sum old, i.e. a cost
  // sT * T on an interval of T.  The iteration then carries c (and n, x) only; NEP_STEP2_FULL=1 keeps the
  // full rows (A/B).
  if (m.step2) {
    const char *e = std::getenv("NEP_STEP2_FULL");
    m.dred = !(e && std::atoi(e) != 0);
    for (int k = 0; k < FN && m.dred; ++k)   // (mf / mt are linear in c only for a binary old allocation)
      m.dred = d.old_allocations[k] == 0.0 || d.old_allocations[k] == 1.0;
    m.sT = m.sigma4 > 0 ? -(m.w_dis - 1.0) : (m.w_dis + 1.0);
    m.sum_old = sum_old;
  }
  m.mem_f.assign(d.function_memory, d.function_memory + F);
  m.node_cost.assign(d.node_cost, d.node_cost + N);
  m.node_budget = d.node_budget;

  // non-x entries of K (COO) and x-row norms (x columns are never rescaled)
  Coo K;
  std::vector<double> xmax(o, 0.0), xsum(o, 0.0);
  std::vector<double> mmax(F, 0.0), msum(F, 0.0);
  for (int r = 0; r < m.R; ++r) {
    mmax[m.row_f[r]] = std::max(mmax[m.row_f[r]], (double)m.row_m[r]);
    msum[m.row_f[r]] += m.row_m[r];
  }
  const double *cpr = d.core_per_req;
  for (int f = 0; f < F; ++f)
    for (int j = 0; j < N; ++j) {
      const int k = f * N + j;
      if (m.fac) {   // C3 and c[f, j] - n[j] <= 0 (the x <= c rows are structured: rhoL, below)
        K.add(dl.o3 + j, il.oc + k, m.mem_f[f]);
        K.add(dl.oQ + k, il.oc + k, 1.0);
        K.add(dl.oQ + k, il.on + j, -1.0);
        continue;
      }
      K.add(dl.o1 + k, il.oc + k, -m.M);
      K.add(dl.o2 + k, il.oc + k, -1.0);
      K.add(dl.o3 + j, il.oc + k, m.mem_f[f]);
      xmax[dl.o1 + k] = xmax[dl.o2 + k] = mmax[f];
      xsum[dl.o1 + k] = xsum[dl.o2 + k] = msum[f];
      if (m.has_n) {
        K.add(dl.o6 + j, il.oc + k, 1.0);
        K.add(dl.o7 + j, il.oc + k, 1.0);
      }
      if (m.step2) {
        K.add(dl.oD1 + k, il.omf + k, 1.0);
        K.add(dl.oD1 + k, il.oc + k, -1.0);
        K.add(dl.oD2 + k, il.omt + k, 1.0);
        K.add(dl.oD2 + k, il.oc + k, 1.0);
        K.add(dl.oD3a, il.oc + k, -1.0);
        K.add(dl.oD3b, il.oc + k, 1.0);
        K.add(dl.oD4, il.oc + k, m.sigma4);
      }
    }
  if (m.fac)
    for (int j = 0; j < N; ++j) {
      K.add(dl.o3 + j, il.on + j, -m.capn[j]);
      K.add(dl.o5 + j, il.on + j, -m.capn[N + j]);
    }
  if (m.has_n && !m.fac)
    for (int j = 0; j < N; ++j) {
      K.add(dl.o6 + j, il.on + j, -m.M);
      K.add(dl.o7 + j, il.on + j, -1.0);
      if (m.step2 && m.score_n_coef != 0.0) K.add(dl.oS, il.on + j, m.score_n_coef);
    }
  if (m.step2) {
    K.add(dl.oD3a, il.oa, -1.0);
    K.add(dl.oD3b, il.od, -1.0);
    K.add(dl.oD4, il.od, 1.0);
    K.add(dl.oD4, il.oa, 1.0);
  }
  for (int r = 0; r < m.R; ++r) {
    const int f = m.row_f[r], src = m.row_src[r];
    for (int j = 0; j < N; ++j) {
      const double w = (double)m.row_w[r] * cpr[(size_t)f * N + j];
      xmax[dl.o5 + j] = std::max(xmax[dl.o5 + j], std::fabs(w));
      xsum[dl.o5 + j] += std::fabs(w);
      if (m.step2 && src >= 0 && m.row_wsc[r] != 0.f) {
        const double s = std::fabs((double)m.row_wsc[r] * D[(size_t)src * N + j]);
        xmax[dl.oS] = std::max(xmax[dl.oS], s);
        xsum[dl.oS] += s;
      }
    }
  }
  // row norms for the relative residual: max(1, |bounds|, max |coef|)
  m.rownorm.assign(o, 1.0);
  for (int k = 0; k < o; ++k) {
    double rn = std::max(1.0, xmax[k]);
    if (std::isfinite(m.lo[k])) rn = std::max(rn, std::fabs(m.lo[k]));
    if (std::isfinite(m.hi[k])) rn = std::max(rn, std::fabs(m.hi[k]));
    m.rownorm[k] = rn;
  }
  for (size_t e = 0; e < K.v.size(); ++e) m.rownorm[K.r[e]] = std::max(m.rownorm[K.r[e]], std::fabs(K.v[e]));
  m.Kr = K.r;
  m.Kc = K.c;
  m.Kv = K.v;
  for (int r = 0; r < m.R; ++r) m.x_cost_free = m.x_cost_free && m.row_wobj[r] == 0.f;
  m.ftot.assign(F, 0.0);
  for (int r = 0; r < m.R; ++r) m.ftot[m.row_f[r]] += m.row_m[r];
  for (size_t k = 0; k < (size_t)N * N && m.x_coef_nonneg; ++k) m.x_coef_nonneg = D[k] >= 0.0;
  for (size_t k = 0; k < (size_t)F * N && m.x_coef_nonneg; ++k)
    m.x_coef_nonneg = m.W[k] >= 0.0 && !(cpr[k] < 0.0);

  // the matrix the iteration runs on: K itself, or (step 2, reduced disruption block) K without the idle
  // rows D1/D2/D3a/D3b and with D4 as the row sum c (coefficient 1 on every c, no a / d): scaling and step
  // size are those of the reduced LP (presolve keeps the reference rows of K)
  Coo Kred;
  if (m.dred) {
    for (size_t e = 0; e < K.v.size(); ++e) {
      const int r = K.r[e], c = K.c[e];
      if ((r >= dl.oD1 && r < dl.oD1 + FN) || (r >= dl.oD2 && r < dl.oD2 + FN) || r == dl.oD3a || r == dl.oD3b) continue;
      if (r == dl.oD4) {
        if (c >= il.oc && c < il.oc + FN) Kred.add(r, c, 1.0);
        continue;
      }
      Kred.add(r, c, K.v[e]);
    }
  }
  const Coo &KS = m.dred ? Kred : K;
  // Ruiz equilibration (10 sweeps, inf-norm) + Pock-Chambolle (alpha = 1) on rows and the
  // non-x columns; x columns keep scale 1 so every routing row stays a plain simplex.
  // facility relaxation: the rows x[r, j] - c[f, j] <= 0 of every routing row r of f (x entry 1, unscaled;
  // c entry -gam_c): one scale per (f, j), and nrow_f entries in c[f, j]'s column
  std::vector<int> nrow_f(F, 0);
  for (int r = 0; r < m.R; ++r) nrow_f[m.row_f[r]] += 1;
  if (m.fac) m.rhoL.assign(FN, 1.0);
  auto ruiz = [&](const Coo &KK, std::vector<double> &rho, std::vector<double> &gam) {
    rho.assign(o, 1.0);
    gam.assign(il.n_int, 1.0);
    std::vector<double> rnL(m.fac ? FN : 0);
    std::vector<double> rn(o), cn(il.n_int);
    for (int sweep = 0; sweep < 11; ++sweep) {
      const bool pc = sweep == 10;
      for (int k = 0; k < o; ++k) rn[k] = pc ? rho[k] * xsum[k] : rho[k] * xmax[k];
      std::fill(cn.begin(), cn.end(), 0.0);
      for (size_t e = 0; e < KK.v.size(); ++e) {
        const double a = std::fabs(rho[KK.r[e]] * KK.v[e] * gam[KK.c[e]]);
        if (pc) { rn[KK.r[e]] += a; cn[KK.c[e]] += a; }
        else { rn[KK.r[e]] = std::max(rn[KK.r[e]], a); cn[KK.c[e]] = std::max(cn[KK.c[e]], a); }
      }
      for (int k = 0; k < (m.fac ? FN : 0); ++k) {
        const double gc = gam[il.oc + k], a = m.rhoL[k] * gc;
        rnL[k] = pc ? m.rhoL[k] * (1.0 + gc) : m.rhoL[k] * std::max(1.0, gc);
        const int f = k / N;
        if (pc) cn[il.oc + k] += nrow_f[f] * a;
        else cn[il.oc + k] = std::max(cn[il.oc + k], a);
      }
      for (int k = 0; k < o; ++k)
        if (rn[k] > 0) rho[k] /= std::sqrt(rn[k]);
      for (int k = 0; k < (m.fac ? FN : 0); ++k)
        if (rnL[k] > 0) m.rhoL[k] /= std::sqrt(rnL[k]);
      for (int k = 0; k < il.n_int; ++k)
        if (cn[k] > 0) gam[k] /= std::sqrt(cn[k]);
    }
  };
  ruiz(KS, m.rho, m.gam);

  m.Ks = KS;   // (the device power iteration, power_device, runs on it after setup_device)
  // ||K̃||_2 by power iteration on K̃ᵀK̃ (structured x part + COO part); nep_model_create runs the same passes on
  // the device (power_device, nep_build.hip) from the same start vector
  if (host_power) {
    std::vector<double> zx((size_t)m.R * N), zs(il.n_int), yv(o), gx((size_t)m.R * N), gs(il.n_int);
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> nd;
    for (auto &t : zx) t = nd(rng);
    for (auto &t : zs) t = nd(rng);
    double lam = 0.0;
    for (int it = 0; it < 60; ++it) {
      double nrm = 0.0;
      for (double t : zx) nrm += t * t;
      for (double t : zs) nrm += t * t;
      nrm = std::sqrt(nrm);
      for (auto &t : zx) t /= nrm;
      for (auto &t : zs) t /= nrm;
      // y = K̃ z
      std::fill(yv.begin(), yv.end(), 0.0);
      for (int r = 0; r < m.R; ++r) {
        const int f = m.row_f[r], src = m.row_src[r];
        const double mr = m.row_m[r], wr = m.row_w[r], sc = m.row_wsc[r];
        const double *xr = &zx[(size_t)r * N];
        double srow = 0.0;
        for (int j = 0; j < N; ++j) {
          if (!m.fac) {
            yv[dl.o1 + f * N + j] += mr * xr[j];
            yv[dl.o2 + f * N + j] += mr * xr[j];
          }
          yv[dl.o5 + j] += wr * cpr[(size_t)f * N + j] * xr[j];
          if (m.step2 && src >= 0 && sc != 0.0) srow += sc * D[(size_t)src * N + j] * xr[j];
        }
        if (m.step2) yv[dl.oS] += srow;
      }
      for (size_t e = 0; e < KS.v.size(); ++e) yv[KS.r[e]] += KS.v[e] * m.gam[KS.c[e]] * zs[KS.c[e]];
      for (int k = 0; k < o; ++k) yv[k] *= m.rho[k];
      // g = K̃ᵀ y
      for (int k = 0; k < o; ++k) yv[k] *= m.rho[k];   // now ρ y
      for (int r = 0; r < m.R; ++r) {
        const int f = m.row_f[r], src = m.row_src[r];
        const double mr = m.row_m[r], wr = m.row_w[r], sc = m.row_wsc[r];
        double *gr = &gx[(size_t)r * N];
        for (int j = 0; j < N; ++j) {
          double g = wr * cpr[(size_t)f * N + j] * yv[dl.o5 + j];
          if (!m.fac) g += mr * (yv[dl.o1 + f * N + j] + yv[dl.o2 + f * N + j]);
          if (m.step2 && src >= 0 && sc != 0.0) g += sc * D[(size_t)src * N + j] * yv[dl.oS];
          gr[j] = g;
        }
      }
      std::fill(gs.begin(), gs.end(), 0.0);
      if (m.fac)   // the x <= c rows, scaled: t = rhoL (x - gam_c z_c); x gets rhoL t, z_c gets -rhoL t (gam_c: below)
        for (int r = 0; r < m.R; ++r) {
          const int f = m.row_f[r];
          const double *xr = &zx[(size_t)r * N];
          double *gr = &gx[(size_t)r * N];
          for (int j = 0; j < N; ++j) {
            const int k = f * N + j;
            const double t = m.rhoL[k] * (xr[j] - m.gam[il.oc + k] * zs[il.oc + k]);
            gr[j] += m.rhoL[k] * t;
            gs[il.oc + k] -= m.rhoL[k] * t;
          }
        }
      for (size_t e = 0; e < KS.v.size(); ++e) gs[KS.c[e]] += KS.v[e] * yv[KS.r[e]];
      for (int k = 0; k < il.n_int; ++k) gs[k] *= m.gam[k];
      double dot = 0.0;
      for (size_t k = 0; k < zx.size(); ++k) dot += zx[k] * gx[k];
      for (int k = 0; k < il.n_int; ++k) dot += zs[k] * gs[k];
      lam = dot;
      zx.swap(gx);
      zs.swap(gs);
    }
    m.sigma_max = std::sqrt(std::max(lam, 1e-30));
    m.eta = 0.95 / m.sigma_max;
    m.power_host = true;
  }

  // initial primal weight (PDLP): ||c~||_2 / ||b~||_2 in the scaled space.  The NEPTUNE objectives
  // are tiny per unit of flow (e.g. (1-alpha) W D / MWD ~ 1e-4, objectives.py:30-52) while the row
  // bounds are node capacities ~1e2, so the balanced weight is far below 1; starting at 1 costs
  // tens of thousands of iterations before the restarts find it.
  {
    double cn2 = 0.0, bn2 = 0.0;
    for (int r = 0; r < m.R; ++r) {
      const int src = m.row_src[r];
      if (src < 0 || m.row_wobj[r] == 0.f) continue;
      for (int j = 0; j < N; ++j) {
        const double cx = (double)m.row_wobj[r] * D[(size_t)src * N + j];
        cn2 += m.row_m[r] * cx * cx;
      }
    }
    for (int k = 0; k < il.n_int; ++k) {
      double ck = m.cost_int[k];
      if (m.dred) {   // the reduced LP's costs at natural bounds: c carries mf / mt (w, -w) and sT; the rest 0
        ck = 0.0;
        if (k >= il.oc && k < il.oc + FN) ck = (d.old_allocations[k - il.oc] > 0.5 ? -m.w_dis : m.w_dis) + m.sT;
        else if (il.on >= 0 && k >= il.on) ck = m.cost_int[k];
      }
      cn2 += std::pow(m.gam[k] * ck, 2);
    }
    for (int k = 0; k < o; ++k) {
      if (m.dred && ((k >= dl.oD1 && k < dl.oD1 + FN) || (k >= dl.oD2 && k < dl.oD2 + FN) || k == dl.oD3a ||
                     k == dl.oD3b))
        continue;   // (idle rows of the reduced LP)
      double b = 0.0;
      if (std::isfinite(m.lo[k])) b = std::max(b, std::fabs(m.lo[k]));
      if (std::isfinite(m.hi[k])) b = std::max(b, std::fabs(m.hi[k]));
      if (m.fac && k >= dl.o3 && k < dl.o5 + N) b = m.capn[k < dl.o5 ? k - dl.o3 : N + k - dl.o5];   // (hi = 0)
      if (m.dred && k == dl.oD4) {   // the row sum c in [L, U] at the natural allocated / deallocated bounds
        double tlo, thi;
        dred_interval(m.sigma4, m.nat_lb[il.oa], m.nat_ub[il.oa], m.nat_lb[il.od], m.nat_ub[il.od], tlo, thi);
        b = std::max(std::fabs(m.sum_old + tlo), std::fabs(m.sum_old + thi));
      }
      bn2 += std::pow(m.rho[k] * b, 2);
    }
    m.omega0 = (cn2 > 0.0 && bn2 > 0.0) ? std::sqrt(cn2) / std::sqrt(bn2) : 1.0;
  }
  return NEP_OK;
}

int setup_device(Model &m, int max_batch, void *stream) {
  m.max_batch = max_batch;
  m.busy.assign(max_batch, 0);
  if (stream) {
    m.stream = (hipStream_t)stream;
  } else {
    HIPCHK(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
    m.own_stream = true;
  }
  HIPCHK(hipEventCreate(&m.ev0));
  HIPCHK(hipEventCreate(&m.ev1));
  // the auxiliary stream (host reads of finished slots, warm-start copies, submits) at the highest priority:
  // its small kernels and copies are dispatched between the workgroups of the block in flight instead of
  // queueing behind it (round-4 B&B profile: a flows read waited ~0.5 ms for a 64x32 block)
  // (NEP_AUX_PRIORITY=0: default priority — the rocprofv3 PMC passes of tools/traffic.py run that way)
  {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
    const char *e = std::getenv("NEP_AUX_PRIORITY");
    if (e && std::atoi(e) == 0) greatest = least;
    HIPCHK(hipStreamCreateWithPriority(&m.aux, hipStreamNonBlocking, greatest));
  }
  HIPCHK(hipEventCreateWithFlags(&m.ev_aux, hipEventDisableTiming));
  DeviceView &v = m.v;
  v.N = m.N; v.NP = m.NP; v.F = m.F; v.R = m.R; v.JB = m.JB; v.CPL = m.CPL;
  v.has_n = m.has_n; v.step2 = m.step2; v.variant = m.variant; v.fac = m.fac;
  v.M = m.M; v.eps = m.eps; v.sigma4 = m.sigma4; v.cost_n = m.cost_n; v.score_n_coef = m.score_n_coef;
  v.w_dis = m.w_dis;
  v.dred = m.dred; v.sT = m.sT; v.sum_old = m.sum_old;
  v.dl = m.dl; v.il = m.il;
  v.rs_suff = 0.2; v.rs_nec = 0.9; v.rs_art = 0.36; v.omega_smooth = 0.5;   // necessary 0.9: DESIGN.md §4
  if (const char *e = std::getenv("NEP_RESTART")) std::sscanf(e, "%lf,%lf,%lf", &v.rs_suff, &v.rs_nec, &v.rs_art);
  if (const char *e = std::getenv("NEP_OMEGA_SMOOTH")) v.omega_smooth = std::atof(e);
  if (const char *e = std::getenv("NEP_PIPELINE_MAX_DONE")) m.pipe_max_done = std::atoi(e);
  v.polish_res = kPolishRes;
  v.polish_budget = kPolishBudget;
  if (const char *e = std::getenv("NEP_POLISH")) {   // "res,budget"
    long long b = v.polish_budget;
    std::sscanf(e, "%lf,%lld", &v.polish_res, &b);
    v.polish_budget = b;
  }
  int rc;
  if ((rc = upload(m, &v.rows, m.rows))) return rc;
  if ((rc = upload(m, &v.frow, m.frow))) return rc;
  if ((rc = upload(m, &v.gam, m.gam))) return rc;
  if ((rc = upload(m, &v.rho, m.rho))) return rc;
  if ((rc = upload(m, &v.lo, m.lo))) return rc;
  if ((rc = upload(m, &v.hi, m.hi))) return rc;
  if ((rc = upload(m, &v.rownorm, m.rownorm))) return rc;
  if ((rc = upload(m, &v.cost_int, m.cost_int))) return rc;
  if ((rc = upload(m, &v.mem_f, m.mem_f))) return rc;
  if ((rc = upload(m, &v.capn, m.capn))) return rc;
  return NEP_OK;
}

int setup_dense(Model &m, const nep_model_desc &d) {
  DeviceView &v = m.v;
  const int N = m.N, NP = m.NP, F = m.F;
  std::vector<float> Dp((size_t)N * NP, 0.f), cp((size_t)F * NP, 0.f);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) Dp[(size_t)i * NP + j] = (float)d.delay[(size_t)i * N + j];
  for (int f = 0; f < F; ++f)
    for (int j = 0; j < N; ++j) {
      double c = d.core_per_req[(size_t)f * N + j];
      if (!std::isfinite(c)) c = std::numeric_limits<float>::max();
      cp[(size_t)f * NP + j] = (float)std::min(c, (double)std::numeric_limits<float>::max());
    }
  int rc;
  if ((rc = upload(m, &v.D, Dp))) return rc;
  if ((rc = upload(m, &v.cpr, cp))) return rc;
  // per-slot arrays
  const int B = m.max_batch;
  v.sx = (int64_t)m.R * NP;
  if (const char *e = std::getenv("NEP_SLOT_PAD")) v.sx += std::max(0, std::atoi(e)) / 64 * 64;   // (probe)
  v.smask = (int64_t)F * NP;
  v.sint = m.il.n_int;
  v.sdual = m.dl.n_dual;
  v.skty = (int64_t)F * NP + NP + 4;
  v.stpart = (int64_t)F * NTS;
  v.sbpart = (int64_t)(F + m.JB) * NBS;
  v.snpart = (int64_t)F * (m.fac ? 3 : 2) * NP;   // fac: c, CPU share, reflected c (2ĉ - c) per (f, j)
  v.srpart = (int64_t)F * 2 * NP;
  {   // (probe: NEP_SLOT_OVERALLOC=k allocates the routing state for k x the slots; only B are used)
    const char *e = std::getenv("NEP_SLOT_OVERALLOC");
    const size_t k = e ? (size_t)std::max(1, std::atoi(e)) : 1;
    if ((rc = dalloc(m, &v.x, k * B * v.sx))) return rc;
    if ((rc = dalloc(m, &v.xa, k * B * v.sx))) return rc;
  }
  if ((rc = dalloc(m, &v.acnt, (size_t)B * m.R))) return rc;
  if ((rc = dalloc(m, &v.aent, (size_t)B * m.R * kAnchorK))) return rc;
  if ((rc = dalloc(m, &v.theta, (size_t)B * m.R))) return rc;
  if ((rc = dalloc(m, &v.mask, (size_t)B * v.smask))) return rc;
  if ((rc = dalloc(m, &v.zi, (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &v.zia, (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &v.zr, (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &v.lb, (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &v.ub, (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &v.y, (size_t)B * v.sdual))) return rc;
  if ((rc = dalloc(m, &v.ya, (size_t)B * v.sdual))) return rc;
  if ((rc = dalloc(m, &v.ybak, (size_t)B * v.sdual))) return rc;
  if ((rc = dalloc(m, &v.kz, (size_t)B * v.sdual))) return rc;
  if ((rc = dalloc(m, &v.kza, (size_t)B * v.sdual))) return rc;
  if ((rc = dalloc(m, &v.kty, (size_t)B * v.skty))) return rc;
  if ((rc = dalloc(m, &v.tpart, (size_t)B * v.stpart))) return rc;
  if ((rc = dalloc(m, &v.bpart, (size_t)B * v.sbpart))) return rc;
  if ((rc = dalloc(m, &v.npart, (size_t)B * v.snpart))) return rc;
  if (m.fac) {
    v.slsum = (int64_t)F * NP;
    if ((rc = dalloc(m, &v.lam, (size_t)B * v.sx))) return rc;
    if ((rc = dalloc(m, &v.lama, (size_t)B * v.sx))) return rc;
    if ((rc = dalloc(m, &v.lsum, (size_t)B * v.slsum))) return rc;
    std::vector<float> rl((size_t)F * NP, 0.f);
    for (int f = 0; f < F; ++f)
      for (int j = 0; j < N; ++j) rl[(size_t)f * NP + j] = (float)m.rhoL[(size_t)f * N + j];
    if ((rc = upload(m, &v.rho_l, rl))) return rc;
    HIPCHK(hipMemsetAsync(v.lam, 0, sizeof(float) * B * v.sx, m.stream));
    HIPCHK(hipMemsetAsync(v.lsum, 0, sizeof(float) * B * v.slsum, m.stream));
  }
  if ((rc = dalloc(m, &v.rpart, (size_t)B * v.srpart))) return rc;
  if ((rc = dalloc(m, &v.ctrl, (size_t)B))) return rc;
  {
    void *h = nullptr;
    if (hipHostMalloc(&h, sizeof(Ctrl) * B) != hipSuccess) return fail(NEP_ERR_NOMEM, "hipHostMalloc (Ctrl)");
    m.h_ctrl = static_cast<Ctrl *>(h);
    if (hipHostMalloc(&h, sizeof(int32_t) * B) != hipSuccess) return fail(NEP_ERR_NOMEM, "hipHostMalloc (act)");
    m.h_act = static_cast<int32_t *>(h);
  }
  if ((rc = dalloc(m, &m.d_prm, 3))) return rc;
  v.prm = m.d_prm;
  if ((rc = dalloc(m, &m.d_slots, (size_t)B))) return rc;
  if ((rc = dalloc(m, &m.d_new, (size_t)B))) return rc;
  {
    const double *p = nullptr;
    if ((rc = upload(m, &p, m.base_lb))) return rc;
    m.d_base_lb = const_cast<double *>(p);
    if ((rc = upload(m, &p, m.base_ub))) return rc;
    m.d_base_ub = const_cast<double *>(p);
    const uint8_t *q = nullptr;
    if ((rc = upload(m, &q, m.base_mask))) return rc;
    m.d_base_mask = const_cast<uint8_t *>(q);
  }
  if ((rc = dalloc(m, &m.d_sub_i, (size_t)3 * B + 1 + (size_t)B * v.sint))) return rc;
  if ((rc = dalloc(m, &m.d_sub_d, (size_t)2 * B * v.sint))) return rc;
  HIPCHK(hipMemsetAsync(v.ctrl, 0, sizeof(Ctrl) * B, m.stream));
  HIPCHK(hipMemsetAsync(v.x, 0, sizeof(float) * B * v.sx, m.stream));
  HIPCHK(hipMemsetAsync(v.xa, 0, sizeof(float) * B * v.sx, m.stream));
  HIPCHK(hipMemsetAsync(v.acnt, 0, sizeof(int32_t) * B * m.R, m.stream));
  HIPCHK(hipMemsetAsync(v.theta, 0xFF, sizeof(float) * B * m.R, m.stream));   // NaN: no hint
  HIPCHK(hipMemsetAsync(v.zi, 0, sizeof(double) * B * v.sint, m.stream));
  HIPCHK(hipMemsetAsync(v.y, 0, sizeof(double) * B * v.sdual, m.stream));
  HIPCHK(hipStreamSynchronize(m.stream));
  return NEP_OK;
}

// The step size on the device (nep_build.hip): the host build's 60 power-iteration passes on K̃ᵀK̃ from the same
// start vector (mt19937_64(12345) normals, routing entries first), in fp64 with fixed-order reductions, over the
// device copies of the rows, delay and core_per_req matrices (fp32, as the iteration reads them) and the CSR / CSC
// of the small-variable part.  Scratch is freed afterwards.
static int power_device(Model &m) {
  const DeviceView &v = m.v;
  const int N = m.N, o = m.dl.n_dual, ni = m.il.n_int;
  const size_t nx = (size_t)m.R * N;
  std::vector<double> zx(nx), zs(ni);
  {
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> nd;
    for (auto &t : zx) t = nd(rng);
    for (auto &t : zs) t = nd(rng);
  }
  const Coo &K = m.Ks;
  const size_t ne = K.v.size();
  std::vector<int32_t> rp(o + 1, 0), ci(ne), cp(ni + 1, 0), ri(ne);
  std::vector<double> cv(ne), rv(ne);
  for (size_t e = 0; e < ne; ++e) { rp[K.r[e] + 1]++; cp[K.c[e] + 1]++; }
  for (int k = 0; k < o; ++k) rp[k + 1] += rp[k];
  for (int k = 0; k < ni; ++k) cp[k + 1] += cp[k];
  {
    std::vector<int32_t> fr(rp.begin(), rp.end() - 1), fc(cp.begin(), cp.end() - 1);
    for (size_t e = 0; e < ne; ++e) {
      const int a = fr[K.r[e]]++, b = fc[K.c[e]]++;
      ci[a] = K.c[e]; cv[a] = K.v[e];
      ri[b] = K.r[e]; rv[b] = K.v[e];
    }
  }
  constexpr int kIters = 60, kBlk = 512;
  std::vector<void *> tmp;
  auto alloc = [&](size_t bytes) -> void * {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 8)) != hipSuccess) return nullptr;
    tmp.push_back(p);
    return p;
  };
  auto release = [&]() { for (void *p : tmp) (void)hipFree(p); tmp.clear(); };
  double *dzx = (double *)alloc(nx * 8), *dgx = (double *)alloc(nx * 8), *dzs = (double *)alloc(ni * 8);
  double *dgs = (double *)alloc(ni * 8), *dy = (double *)alloc((size_t)o * 8);
  double *dup = (double *)alloc((size_t)m.F * N * 8), *dsp = (double *)alloc((size_t)m.F * 8);
  double *dgf = (double *)alloc((size_t)m.F * N * 8), *dpart = (double *)alloc(kBlk * 8);
  double *dout = (double *)alloc((kIters + 1) * 8);
  int32_t *drp = (int32_t *)alloc((o + 1) * 4), *dci = (int32_t *)alloc(ne * 4), *dcp = (int32_t *)alloc((ni + 1) * 4);
  int32_t *dri = (int32_t *)alloc(ne * 4);
  double *dcv = (double *)alloc(ne * 8), *drv = (double *)alloc(ne * 8);
  for (void *p : tmp)
    if (!p) { release(); return fail(NEP_ERR_NOMEM, "hipMalloc (device power iteration)"); }
  hipError_t e = hipSuccess;
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  if (e == hipSuccess) e = hipMemcpyAsync(dzx, zx.data(), nx * 8, h2d, m.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dzs, zs.data(), (size_t)ni * 8, h2d, m.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(drp, rp.data(), rp.size() * 4, h2d, m.stream);
  if (e == hipSuccess && ne) e = hipMemcpyAsync(dci, ci.data(), ne * 4, h2d, m.stream);
  if (e == hipSuccess && ne) e = hipMemcpyAsync(dcv, cv.data(), ne * 8, h2d, m.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dcp, cp.data(), cp.size() * 4, h2d, m.stream);
  if (e == hipSuccess && ne) e = hipMemcpyAsync(dri, ri.data(), ne * 4, h2d, m.stream);
  if (e == hipSuccess && ne) e = hipMemcpyAsync(drv, rv.data(), ne * 8, h2d, m.stream);
  if (e == hipSuccess)
    e = launch_power_iteration(v, kIters, dzx, dzs, dgx, dgs, dy, dup, dsp, dgf, dpart, kBlk, dout, drp, dci, dcv, dcp,
                               dri, drv, m.stream);
  double lam = 0.0;
  if (e == hipSuccess) e = hipMemcpyAsync(&lam, dout + kIters, 8, hipMemcpyDeviceToHost, m.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(m.stream);
  release();
  if (e != hipSuccess) return fail(NEP_ERR_HIP, std::string("device power iteration: ") + hipGetErrorString(e));
  m.sigma_max = std::sqrt(std::max(lam, 1e-30));
  m.eta = 0.95 / m.sigma_max;
  m.power_host = false;
  return NEP_OK;
}

// Node presolve: bounds, the C8 cap, n_ub = 0 => c_ub[:, j] = 0, destination masks, and a
// row-activity test over the node's box: the activity range of each dualised row, from the small
// variables' bounds and the x part's range (flow into (f, j) is in [0, ftot_f] when j is allowed for
// f, else 0; the CPU and score rows have non-negative x coefficients).  A row whose range misses
// [lo, hi] proves the node LP infeasible — e.g. step-2 delete mode with more fixed placements than
// the old allocation (constraints_step2.py:36-44), memory over-committed by fixed placements
// (constraints_step1.py:18-23), an open node with every placement closed (:69-78).
//
// presolve_full() evaluates all of it from scratch; it runs once per model on the natural bounds
// (the "base" box).  presolve_node() evaluates a node as a sparse change of that base: node bounds
// only tighten the base box, so a base-infeasible model makes every node infeasible, rows no
// changed variable touches keep their (feasible) base range, and the rows a change touches are
// re-tested from base range + delta (CSC of the non-x part of K).  Cost per node: one O(n_int) scan
// of the caller's bounds + O(changes x column length), instead of O(n_int + nnz(K) + F*N).
static void activity_ranges(const Model &m, const std::vector<double> &lb, const std::vector<double> &ub,
                            const std::vector<uint8_t> &mask, std::vector<double> &amin, std::vector<double> &amax) {
  const int N = m.N, F = m.F, NP = m.NP, o = m.dl.n_dual;
  amin.assign(o, 0.0);
  amax.assign(o, 0.0);
  for (int f = 0; f < F && m.dl.o1 >= 0; ++f)   // (C1/C2: not in the facility relaxation)
    for (int j = 0; j < N; ++j) {
      const double fx = mask[(size_t)f * NP + j] ? m.ftot[f] : 0.0;
      amax[m.dl.o1 + f * N + j] += fx;
      amax[m.dl.o2 + f * N + j] += fx;
    }
  for (int j = 0; j < N; ++j) {
    amax[m.dl.o5 + j] = INF;
    if (!m.x_coef_nonneg) amin[m.dl.o5 + j] = -INF;
  }
  if (m.step2) {
    amax[m.dl.oS] = INF;
    if (!m.x_coef_nonneg) amin[m.dl.oS] = -INF;
  }
  for (size_t e = 0; e < m.Kv.size(); ++e) {
    const double a = m.Kv[e] * lb[m.Kc[e]], b = m.Kv[e] * ub[m.Kc[e]];
    amin[m.Kr[e]] += std::min(a, b);
    amax[m.Kr[e]] += std::max(a, b);
  }
}

static inline bool row_range_ok(const Model &m, int k, double amin, double amax) {
  if (amin > m.hi[k] + 1e-9 * std::max(1.0, std::fabs(m.hi[k]))) return false;
  if (amax < m.lo[k] - 1e-9 * std::max(1.0, std::fabs(m.lo[k]))) return false;
  return true;
}

// the step-2 score / delay row's smallest activity over the routing simplexes: sum_r wsc[r] min over
// the allowed destinations j of f_r of D[src_r, j] (allow: [F][ld] nonzero = allowed)
static double score_row_xmin(const Model &m, const uint8_t *allow, int ld) {
  const int N = m.N;
  double xmin = 0.0;
  for (int r = 0; r < m.R; ++r) {
    const double w = m.row_wsc_d[r];   // fp64: a proof of infeasibility must not rest on fp32 rounding
    if (w == 0.0) continue;
    const double *Dr = &m.Dh[(size_t)m.row_src[r] * N];
    const uint8_t *al = allow + (size_t)m.row_f[r] * ld;
    double mn = INF;
    for (int j = 0; j < N; ++j)
      if (al[j]) mn = std::min(mn, Dr[j]);
    if (mn < INF) xmin += w * mn;
  }
  return xmin;
}

// CPU cover test over a box's allowed placements allow[f * ld + j] (c[f, j] not fixed to 0): every routing
// row of f sends its whole workload W[f, i] to allowed destinations (C4, constraints_step1.py:27-34), each
// unit costing cpr[f, j] cores at j (C5, :57-65), so (a) sum_f wsum_f min_{j allowed} cpr[f, j] cannot exceed
// the cores of the nodes any loaded function may use, and (b) a function with ONE allowed destination puts
// all of wsum_f cpr[f, j] on that node.  Either failing proves the box infeasible — e.g. a rounding leaf
// that opens too few nodes, whose LP PDHG can only stall on (a residual stuck at the overload).  Only for
// non-negative CPU coefficients (the generator's and the reference's inputs).
static bool cpu_cover_ok(const Model &m, const uint8_t *allow, int ld) {
  if (!m.x_coef_nonneg) return true;
  const int N = m.N, F = m.F;
  std::vector<uint8_t> usable(N, 0);
  std::vector<double> forced(N, 0.0);
  double demand = 0.0;
  for (int f = 0; f < F; ++f) {
    if (m.wsum[f] <= 0.0) continue;
    const uint8_t *al = allow + (size_t)f * ld;
    double mc = INF;
    int cnt = 0, only = -1;
    for (int j = 0; j < N; ++j)
      if (al[j]) {
        mc = std::min(mc, m.cprh[(size_t)f * N + j]);
        usable[j] = 1;
        ++cnt;
        only = j;
      }
    if (cnt == 0) return false;
    demand += m.wsum[f] * mc;
    if (cnt == 1) forced[only] += m.wsum[f] * m.cprh[(size_t)f * N + only];
  }
  double cap = 0.0;
  for (int j = 0; j < N; ++j) {
    const double cores = m.capn[N + j];
    if (forced[j] > cores + 1e-6 * std::max(1.0, cores)) return false;
    if (usable[j]) cap += cores;
  }
  return demand <= cap + 1e-6 * std::max(1.0, cap);
}

bool presolve_full(const Model &m, const double *lbi, const double *ubi, std::vector<double> &lb,
                   std::vector<double> &ub, std::vector<uint8_t> &mask) {
  const int n = m.il.n_int, N = m.N, F = m.F, NP = m.NP;
  lb = m.nat_lb;
  ub = m.nat_ub;
  if (lbi)
    for (int k = 0; k < n; ++k) lb[k] = std::max(lb[k], lbi[k]);
  if (ubi)
    for (int k = 0; k < n; ++k) ub[k] = std::min(ub[k], ubi[k]);
  if (m.step2)   // (see presolve_node: c within the box its moved_from / moved_to bounds imply)
    for (int k = 0; k < F * N; ++k) {
      const double old = -m.lo[m.dl.oD1 + k];
      ub[m.il.oc + k] = std::min(ub[m.il.oc + k], old + ub[m.il.omf + k]);
      lb[m.il.oc + k] = std::max(lb[m.il.oc + k], old - ub[m.il.omt + k]);
    }
  bool ok = true;
  if (m.has_n)
    for (int j = 0; j < N; ++j)
      if (ub[m.il.on + j] <= 0.0)
        for (int f = 0; f < F; ++f) ub[m.il.oc + f * N + j] = std::min(ub[m.il.oc + f * N + j], 0.0);
  for (int k = 0; k < n; ++k)
    if (lb[k] > ub[k] + 1e-12) ok = false;
  mask.assign((size_t)F * NP, 0);
  for (int f = 0; f < F; ++f) {
    int cnt = 0;
    for (int j = 0; j < N; ++j) {
      const bool a = ub[m.il.oc + f * N + j] > 0.0;
      mask[(size_t)f * NP + j] = a;
      cnt += a;
    }
    if (cnt == 0) ok = false;   // every routing row of f would be empty (C4 infeasible)
  }
  if (!ok) return false;
  std::vector<double> amin, amax;
  activity_ranges(m, lb, ub, mask, amin, amax);
  if (m.score_x) amin[m.dl.oS] += score_row_xmin(m, mask.data(), NP);   // (see presolve_node)
  for (int k = 0; k < m.dl.n_dual; ++k)
    if (!row_range_ok(m, k, amin[k], amax[k])) return false;
  return cpu_cover_ok(m, mask.data(), NP);
}

static void init_scratch(const Model &m, PresolveScratch &s) {
  s.pos.assign(m.il.n_int, -1);
  s.dmin.assign(m.dl.n_dual, 0.0);
  s.dmax.assign(m.dl.n_dual, 0.0);
  s.rowmark.assign(m.dl.n_dual, 0);
  s.fdelta.assign(m.F, 0);
  s.allow.assign((size_t)m.F * m.N, 0);
}

// once per model: the base box (natural bounds) and what presolve_node() needs
void presolve_setup(Model &m) {
  const int n = m.il.n_int, F = m.F, NP = m.NP;
  m.base_ok = presolve_full(m, nullptr, nullptr, m.base_lb, m.base_ub, m.base_mask);
  activity_ranges(m, m.base_lb, m.base_ub, m.base_mask, m.base_amin, m.base_amax);
  m.base_cnt.assign(F, 0);
  for (int f = 0; f < F; ++f)
    for (int j = 0; j < m.N; ++j) m.base_cnt[f] += m.base_mask[(size_t)f * NP + j];
  m.Kcp.assign(n + 1, 0);
  for (int c : m.Kc) m.Kcp[c + 1]++;
  for (int k = 0; k < n; ++k) m.Kcp[k + 1] += m.Kcp[k];
  m.Kcr.resize(m.Kc.size());
  m.Kcv.resize(m.Kc.size());
  std::vector<int> fill(m.Kcp.begin(), m.Kcp.end() - 1);
  for (size_t e = 0; e < m.Kc.size(); ++e) {
    const int at = fill[m.Kc[e]]++;
    m.Kcr[at] = m.Kr[e];
    m.Kcv[at] = m.Kv[e];
  }
  m.psc.resize(1);
  init_scratch(m, m.psc[0]);
}

// One node as changes (index, lb, ub) of the base box, appended to ci/cl/cu.  Returns false (and
// appends nothing) if the node is infeasible.
bool presolve_node(const Model &m, PresolveScratch &sc, const double *lbi, const double *ubi, std::vector<int32_t> &ci,
                   std::vector<double> &cl, std::vector<double> &cu) {
  const int n = m.il.n_int, N = m.N, F = m.F, NP = m.NP, oc = m.il.oc;
  if (!m.base_ok) return false;
  const size_t c0 = ci.size();
  for (int k = 0; k < n; ++k) {
    const double l = lbi ? std::max(m.base_lb[k], lbi[k]) : m.base_lb[k];
    const double u = ubi ? std::min(m.base_ub[k], ubi[k]) : m.base_ub[k];
    if (l != m.base_lb[k] || u != m.base_ub[k]) {
      sc.pos[k] = (int)(ci.size() - c0);
      ci.push_back(k);
      cl.push_back(l);
      cu.push_back(u);
    }
  }
  if (m.step2) {
    // bound propagation through the disruption rows D1 / D2 (constraints_step2.py:5-16): mf - c >= -old and
    // mt + c >= old give c <= old + ub(mf) and c >= old - ub(mt).  A node that fixes moved_from = 0 where
    // old = 0 closes the placement — so its routing column is masked, instead of PDHG having to find that its
    // flow must be 0 through the 1/M-priced big-M row (payload.json step 2: 1.4 units of flow left on such a
    // column after 200k iterations)
    const size_t nc = ci.size();
    for (size_t t = c0; t < nc; ++t) {
      const int k = ci[t];
      const bool isf = k >= m.il.omf && k < m.il.omf + F * N, ist = k >= m.il.omt && k < m.il.omt + F * N;
      if (!isf && !ist) continue;
      const int q = k - (isf ? m.il.omf : m.il.omt);
      const double old = -m.lo[m.dl.oD1 + q];
      const int kc = oc + q;
      double nl = -INF, nu = INF;
      if (isf) nu = old + cu[t];
      else nl = old - cu[t];
      if (sc.pos[kc] >= 0) {
        const size_t pc = c0 + sc.pos[kc];
        cu[pc] = std::min(cu[pc], nu);
        cl[pc] = std::max(cl[pc], nl);
      } else if (nu < m.base_ub[kc] || nl > m.base_lb[kc]) {
        sc.pos[kc] = (int)(ci.size() - c0);
        ci.push_back(kc);
        cl.push_back(std::max(m.base_lb[kc], nl));
        cu.push_back(std::min(m.base_ub[kc], nu));
      }
    }
  }
  if (m.has_n) {
    const size_t nc = ci.size();
    for (size_t t = c0; t < nc; ++t) {
      const int k = ci[t];
      if (k < m.il.on || k >= m.il.on + N || cu[t] > 0.0) continue;
      const int j = k - m.il.on;
      for (int f = 0; f < F; ++f) {
        const int kc = oc + f * N + j;
        if (sc.pos[kc] >= 0) {
          double &u = cu[c0 + sc.pos[kc]];
          u = std::min(u, 0.0);
        } else if (m.base_ub[kc] > 0.0) {
          sc.pos[kc] = (int)(ci.size() - c0);
          ci.push_back(kc);
          cl.push_back(m.base_lb[kc]);
          cu.push_back(0.0);
        }
      }
    }
  }
  bool ok = true;
  std::vector<int> &touched = sc.touched, &ftouched = sc.ftouched;
  touched.clear();
  ftouched.clear();
  // a node that changes many variables (a rounding leaf fixes every c and n) re-tests every row instead of
  // tracking the touched ones: the bookkeeping costs more than the test
  const bool dense = (ci.size() - c0) * 8 > (size_t)m.dl.n_dual;
  auto touch = [&](int r) {
    if (!dense && !sc.rowmark[r]) { sc.rowmark[r] = 1; touched.push_back(r); }
  };
  {
    // (raw pointers: the loop streams the CSC of K, ~7 row updates per change)
    const int *Kcp = m.Kcp.data(), *Kcr = m.Kcr.data();
    const double *Kcv = m.Kcv.data(), *blo = m.base_lb.data(), *bup = m.base_ub.data(), *ftot = m.ftot.data();
    const uint8_t *bmask = m.base_mask.data();
    double *dmin = sc.dmin.data(), *dmax = sc.dmax.data();
    int *fdelta = sc.fdelta.data();
    const int32_t *cip = ci.data();
    const double *clp = cl.data(), *cup = cu.data();
    const int o1 = m.dl.o1, o2 = m.dl.o2, FN = F * N;
    const size_t nchg = ci.size();
    for (size_t t = c0; t < nchg; ++t) {
      const int k = cip[t];
      const double l = clp[t], u = cup[t];
      if (l > u + 1e-12) ok = false;
      if (k >= oc && k < oc + FN) {
        const int q = k - oc, f = q / N, j = q - f * N;
        const int now = u > 0.0, was = bmask[(size_t)f * NP + j];
        if (now != was) {
          if (fdelta[f] == 0) ftouched.push_back(f);
          fdelta[f] += now - was;
          if (o1 >= 0) {   // (C1/C2: not in the facility relaxation)
            const double dfx = (now - was) * ftot[f];
            touch(o1 + q);
            touch(o2 + q);
            dmax[o1 + q] += dfx;
            dmax[o2 + q] += dfx;
          }
        }
      }
      const double bl = blo[k], bu = bup[k];
      for (int e = Kcp[k]; e < Kcp[k + 1]; ++e) {
        const int r = Kcr[e];
        const double a = Kcv[e];
        touch(r);
        dmin[r] += std::min(a * l, a * u) - std::min(a * bl, a * bu);
        dmax[r] += std::max(a * l, a * u) - std::max(a * bl, a * bu);
      }
    }
  }
  const bool cover = ok && !ftouched.empty();
  if (cover || (ok && m.score_x)) {
    // the node's allowed placements: the base mask with the node's c changes over it
    for (int f = 0; f < F; ++f)
      std::memcpy(&sc.allow[(size_t)f * N], &m.base_mask[(size_t)f * NP], (size_t)N);
    for (size_t t = c0; t < ci.size(); ++t) {
      const int k = ci[t];
      if (k >= oc && k < oc + F * N) sc.allow[k - oc] = cu[t] > 0.0;
    }
  }
  // the CPU cover test (cpu_cover_ok) over the node's allowed placements; a box that closes no placement
  // has the base box's (tested in presolve_full)
  if (cover) ok = cpu_cover_ok(m, sc.allow.data(), N);
  if (ok && m.score_x) {
    // The score / delay row (constraints_step2.py:57-88) over x: every routing row carries mass 1 on its
    // allowed destinations, so its activity is at least sum_r wsc[r] min_{j allowed} D[src_r, j].  Closed
    // placements can push that above the right-hand side (e.g. a step-1 delay of 0 admits only local
    // serving): such a node is infeasible, which PDHG cannot prove (DESIGN.md §4 "Infeasibility").
    const int rs = m.dl.oS;
    touch(rs);
    sc.dmin[rs] += score_row_xmin(m, sc.allow.data(), N);
  }
  for (int f : ftouched) {
    if (m.base_cnt[f] + sc.fdelta[f] == 0) ok = false;   // every routing row of f empty
    sc.fdelta[f] = 0;
  }
  if (dense) {
    for (int r = 0; r < m.dl.n_dual; ++r)
      if (ok && !row_range_ok(m, r, m.base_amin[r] + sc.dmin[r], m.base_amax[r] + sc.dmax[r])) ok = false;
    std::fill(sc.dmin.begin(), sc.dmin.end(), 0.0);
    std::fill(sc.dmax.begin(), sc.dmax.end(), 0.0);
  } else {
    for (int r : touched) {
      if (ok && !row_range_ok(m, r, m.base_amin[r] + sc.dmin[r], m.base_amax[r] + sc.dmax[r])) ok = false;
      sc.dmin[r] = sc.dmax[r] = 0.0;
      sc.rowmark[r] = 0;
    }
  }
  for (size_t t = c0; t < ci.size(); ++t) sc.pos[ci[t]] = -1;
  if (!ok) {
    ci.resize(c0);
    cl.resize(c0);
    cu.resize(c0);
  }
  return ok;
}

nep_lp_opts resolve_opts(const nep_lp_opts *opts) {
  nep_lp_opts o{};
  o.tol = 1e-7;
  o.cutoff = INF;
  o.max_iters = 200000;
  o.check_every = 64;
  o.warm_start = 0;
  o.warm_omega_floor = 2.0;
  o.warm_omega_cap = 4.0;
  if (opts) {
    if (opts->tol > 0) o.tol = opts->tol;
    o.cutoff = opts->cutoff;
    if (opts->max_iters > 0) o.max_iters = opts->max_iters;
    if (opts->check_every > 0) o.check_every = opts->check_every;
    o.warm_start = opts->warm_start;
    if (opts->warm_omega_floor != 0) o.warm_omega_floor = opts->warm_omega_floor < 0 ? 0.0 : opts->warm_omega_floor;
    o.gap_tol = opts->gap_tol;
    if (opts->warm_omega_cap != 0) o.warm_omega_cap = opts->warm_omega_cap < 0 ? 0.0 : opts->warm_omega_cap;
    o.polish_after = opts->polish_after;
    o.bound_res = opts->bound_res > 0 ? opts->bound_res : 0.0;
  }
  if (!(o.gap_tol > 0)) o.gap_tol = o.tol;
  // polishing: by default only warm-started LPs (B&B children) polish; a cold LP (a root) iterates on
  // to its own certificate, whose more converged duals its children then start from
  if (o.polish_after == 0) o.polish_after = o.warm_start ? 256.0 : -1.0;
  return o;
}

// tol / cutoff / gap tol of every LP in flight (device memory, read by the graph-replayed blocks): copied on
// the auxiliary stream when they change
static hipError_t set_prm(Model &m, double tol, double cutoff, double gap_tol) {
  if (m.prm_sent && m.prm_host[0] == tol && m.prm_host[1] == cutoff && m.prm_host[2] == gap_tol) return hipSuccess;
  m.prm_host[0] = tol;
  m.prm_host[1] = cutoff;
  m.prm_host[2] = gap_tol;
  m.prm_sent = true;
  return hipMemcpyAsync(m.d_prm, m.prm_host, sizeof(m.prm_host), hipMemcpyHostToDevice, m.aux);
}

// presolve threads for a submit of n nodes: NEP_PRESOLVE_THREADS (default 8, 1 = serial), only for large
// models (below ~8k integer variables a node presolves in tens of microseconds, less than a thread start)
static int presolve_threads(const Model &m, int n) {
  static const int cap = [] {
    const char *e = std::getenv("NEP_PRESOLVE_THREADS");
    const int v = e ? std::atoi(e) : 8;
    const int hw = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(v, hw > 0 ? hw : 1));
  }();
  if (n < 2 || m.il.n_int < 8192) return 1;
  return std::min(cap, n);
}

// one presolved node box: its changes of the base box (m.psc[t].ci/cl/cu [off, off + cnt)), feasibility and
// whether it fixes the objective
struct NodeBox {
  int t = 0;
  size_t off = 0, cnt = 0;
  bool ok = false, ex = false;
  bool bad = false;   // reduced step 2: a fractional moved_from / moved_to bound (not representable)
};

// Presolve n nodes on the host — over the nodes in parallel when they are large (a rounding leaf at
// 256x128 changes ~33k bounds, ~1 ms of work; presolve_threads) — into box[0 .. n-1].
static void presolve_batch(Model &m, int n, const double *lbi, const double *ubi, std::vector<NodeBox> &box) {
  const size_t ni = (size_t)m.il.n_int;
  box.assign(n, NodeBox{});
  auto one = [&](int b, int t) {
    PresolveScratch &sc = m.psc[t];
    NodeBox &nb = box[b];
    const double *L = lbi ? lbi + (size_t)b * ni : nullptr, *U = ubi ? ubi + (size_t)b * ni : nullptr;
    nb.t = t;
    nb.off = sc.ci.size();
    nb.ok = presolve_node(m, sc, L, U, sc.ci, sc.cl, sc.cu);
    nb.cnt = sc.ci.size() - nb.off;
    // the box fixes the objective when the routing carries no cost and every c and n is fixed (a
    // leaf): mf / mt / allocated / deallocated then follow from c at their cheapest (the repair)
    bool ex = nb.ok && m.x_cost_free && !m.fac;
    const int n_fix_end = m.has_n ? m.il.on + m.N : m.il.oc + m.F * m.N;
    for (int k = m.il.oc; ex && k < m.il.oc + m.F * m.N; ++k)
      ex = L && U && std::max(L[k], m.nat_lb[k]) == std::min(U[k], m.nat_ub[k]);
    for (int k = m.has_n ? m.il.on : n_fix_end; ex && k < n_fix_end; ++k)
      ex = L && U && std::max(L[k], m.nat_lb[k]) == std::min(U[k], m.nat_ub[k]);
    nb.ex = ex;
    if (nb.ok && m.dred) {
      // the reduced disruption block needs integral moved_from / moved_to bounds (binaries: every B&B box
      // has them) and a non-empty interval of T = sum c - sum old (dred_interval)
      const IntLayout &il = m.il;
      const int FN = m.F * m.N;
      double la = m.base_lb[il.oa], ua = m.base_ub[il.oa], ld = m.base_lb[il.od], ud = m.base_ub[il.od];
      for (size_t q = nb.off; q < nb.off + nb.cnt; ++q) {
        const int k = sc.ci[q];
        if (k >= il.omf && k < il.omt + FN) {
          if (std::floor(sc.cl[q]) != sc.cl[q] || std::floor(sc.cu[q]) != sc.cu[q]) nb.bad = true;
        } else if (k == il.oa) {
          la = sc.cl[q]; ua = sc.cu[q];
        } else if (k == il.od) {
          ld = sc.cl[q]; ud = sc.cu[q];
        }
      }
      double tlo, thi;
      dred_interval(m.sigma4, la, ua, ld, ud, tlo, thi);
      if (tlo > thi) nb.ok = false;
    }
  };
  const int nt = presolve_threads(m, n);
  while ((int)m.psc.size() < nt) {
    m.psc.emplace_back();
    init_scratch(m, m.psc.back());
  }
  for (int t = 0; t < nt; ++t) {
    m.psc[t].ci.clear();
    m.psc[t].cl.clear();
    m.psc[t].cu.clear();
  }
  if (nt <= 1) {
    for (int b = 0; b < n; ++b) one(b, 0);
  } else {
    std::atomic<int> next{0};
    auto work = [&](int t) {
      for (int b; (b = next.fetch_add(1)) < n;) one(b, t);
    };
    std::vector<std::thread> th;
    try {
      for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    } catch (const std::system_error &) {   // (fewer threads: this one drains the rest)
    }
    work(0);
    for (auto &t : th) t.join();
  }
}

// Start n node LPs: presolve each on the host, upload its bounds and destination mask, initialise
// the slot (cold or warm) and add it to the iterating set.  status[b] = NEP_LP_INFEASIBLE for a
// node presolve proves infeasible (it does not iterate), else NEP_LP_ITERATION_LIMIT.
int submit(Model &m, int n, const int32_t *slots, const double *lbi, const double *ubi, const nep_lp_opts *opts,
           int32_t *status, const int64_t *mi_per = nullptr, const double *br_per = nullptr) {
  if (n <= 0) return NEP_OK;
  const nep_lp_opts o = resolve_opts(opts);
  if (!m.act.empty() && o.check_every != m.run.check_every)
    return fail(NEP_ERR_STATE, "check_every cannot change while LPs are iterating");
  for (int b = 0; b < n; ++b) {
    const int s = slots[b];
    if (s < 0 || s >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
    if (m.busy[s]) return fail(NEP_ERR_STATE, "slot " + std::to_string(s) + " is still iterating");
  }
  m.run = o;
  DeviceView &v = m.v;
  v.warm_omega_floor = o.warm_omega_floor;
  v.warm_omega_cap = o.warm_omega_cap;
  v.warm_omega_ref = m.omega_ref;
  v.polish_after = (o.polish_after < 0 || m.fac) ? -1 : (int64_t)o.polish_after;   // (fac: no polishing)
  v.max_iters = o.max_iters;
  v.bound_res = o.bound_res;
  // tol / cutoff of every LP in flight: device memory, read by the (graph-replayed) blocks
  HIPCHK(set_prm(m, o.tol, o.cutoff, o.gap_tol));
  std::vector<NodeBox> box;
  const auto tp0 = std::chrono::steady_clock::now();
  presolve_batch(m, n, lbi, ubi, box);
  if (m.prof) {
    m.pr_pre += std::chrono::duration<double>(std::chrono::steady_clock::now() - tp0).count();
    ++m.pr_calls;
    m.pr_lps += n;
  }
  struct StageTimer {   // (the rest of the call: staging and launches)
    Model &m;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    ~StageTimer() {
      if (m.prof) m.pr_stage += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    }
  } stage_timer{m};
  for (int b = 0; b < n; ++b)
    if (box[b].bad)
      return fail(NEP_ERR_ARG, "step-2 node box " + std::to_string(b) +
                               ": moved_from / moved_to bounds must be integral (binary variables; NEP_STEP2_FULL=1 "
                               "iterates the full disruption rows)");
  std::vector<int32_t> fresh, off(1, 0), exact;
  std::vector<double> per_mi, per_br;   // (nep_lp_submit_ex: the fresh slots' own budget / bound stop)
  const bool per = mi_per != nullptr || br_per != nullptr;
  int max_chg = 0;
  for (int b = 0; b < n; ++b) {
    const int s = slots[b];
    const NodeBox &nb = box[b];
    status[b] = nb.ok ? NEP_LP_ITERATION_LIMIT : NEP_LP_INFEASIBLE;
    if (!nb.ok) continue;
    m.busy[s] = 1;
    fresh.push_back(s);
    exact.push_back(nb.ex ? 1 : 0);
    off.push_back(off.back() + (int32_t)nb.cnt);
    max_chg = std::max(max_chg, (int)nb.cnt);
    if (per) {
      per_mi.push_back((double)(mi_per && mi_per[b] > 0 ? mi_per[b] : o.max_iters));
      per_br.push_back(br_per ? (br_per[b] > 0 ? br_per[b] : 0.0) : o.bound_res);
    }
  }
  const size_t nchg = (size_t)off.back();
  if (fresh.empty()) {
    HIPCHK(hipStreamSynchronize(m.aux));
    return NEP_OK;
  }
  const int nf = (int)fresh.size();
  // the node boxes on the device: base box copy + the packed changes scattered over it (a few
  // KB per node instead of the 2 x 8 x n_int bytes of bounds and the F x NP mask), staged through pinned
  // host memory so the call need not wait for the copies (nor for the initialisation kernels behind them)
  const size_t need_i = 2 * (size_t)nf + off.size() + nchg, need_d = 2 * nchg + (per ? 2 * (size_t)nf : 0);
  const int sk = m.sub_k;
  m.sub_k ^= 1;
  if (m.sub_pending[sk]) HIPCHK(hipEventSynchronize(m.ev_sub[sk]));   // that staging's copies have read it
  m.sub_pending[sk] = false;
  if (need_i > m.cap_sub_i[sk]) {
    if (m.h_sub_i[sk]) HIPCHK(hipHostFree(m.h_sub_i[sk]));
    m.h_sub_i[sk] = nullptr;
    m.cap_sub_i[sk] = std::max(need_i, 2 * m.cap_sub_i[sk]);
    void *h = nullptr;
    if (hipHostMalloc(&h, m.cap_sub_i[sk] * sizeof(int32_t)) != hipSuccess) return fail(NEP_ERR_NOMEM, "hipHostMalloc (submit)");
    m.h_sub_i[sk] = static_cast<int32_t *>(h);
  }
  if (need_d > m.cap_sub_d[sk]) {
    if (m.h_sub_d[sk]) HIPCHK(hipHostFree(m.h_sub_d[sk]));
    m.h_sub_d[sk] = nullptr;
    m.cap_sub_d[sk] = std::max(need_d, 2 * m.cap_sub_d[sk]);
    void *h = nullptr;
    if (hipHostMalloc(&h, m.cap_sub_d[sk] * sizeof(double)) != hipSuccess) return fail(NEP_ERR_NOMEM, "hipHostMalloc (submit)");
    m.h_sub_d[sk] = static_cast<double *>(h);
  }
  if (!m.ev_sub[sk]) HIPCHK(hipEventCreateWithFlags(&m.ev_sub[sk], hipEventDisableTiming));
  int32_t *hf = m.h_sub_i[sk], *ho = hf + nf, *hc = ho + off.size(), *he = hc + nchg;
  double *hl = m.h_sub_d[sk], *hu = hl + nchg;
  if (per) {
    std::copy(per_mi.begin(), per_mi.end(), hu + nchg);
    std::copy(per_br.begin(), per_br.end(), hu + nchg + nf);
  }
  std::copy(fresh.begin(), fresh.end(), hf);
  std::copy(off.begin(), off.end(), ho);
  std::copy(exact.begin(), exact.end(), he);
  for (int b = 0, q = 0; b < n; ++b) {   // the feasible nodes' changes, in batch order
    const NodeBox &nb = box[b];
    if (!nb.ok) continue;
    const PresolveScratch &sc = m.psc[nb.t];
    std::memcpy(hc + off[q], sc.ci.data() + nb.off, nb.cnt * sizeof(int32_t));
    std::memcpy(hl + off[q], sc.cl.data() + nb.off, nb.cnt * sizeof(double));
    std::memcpy(hu + off[q], sc.cu.data() + nb.off, nb.cnt * sizeof(double));
    ++q;
  }
  HIPCHK(hipMemcpyAsync(m.d_sub_i, hf, need_i * sizeof(int32_t), hipMemcpyHostToDevice, m.aux));
  if (need_d) HIPCHK(hipMemcpyAsync(m.d_sub_d, hl, need_d * sizeof(double), hipMemcpyHostToDevice, m.aux));
  int32_t *dn = m.d_sub_i, *doff = dn + nf, *didx = doff + off.size(), *dex = didx + nchg;
  double *dlb = m.d_sub_d, *dub = dlb + nchg;
  // the staging is free again once these copies are done (the next submit waits for this event only, not
  // for the initialisation kernels below)
  HIPCHK(hipEventRecord(m.ev_sub[sk], m.aux));
  HIPCHK(launch_node_bounds(v, dn, nf, m.d_base_lb, m.d_base_ub, m.d_base_mask, doff, didx, dlb, dub, max_chg,
                            m.aux));
  HIPCHK(launch_init_slot(v, dn, dex, nf, o.warm_start != 0, m.eta, m.omega0, per ? dub + nchg : nullptr, m.aux));
  HIPCHK(launch_x_pass(v, dn, nf, false, true, true, true, 0, m.aux));
  HIPCHK(launch_node_pass(v, dn, nf, false, true, true, true, 0, m.aux));
  HIPCHK(launch_scalar_pass(v, dn, nf, false, true, true, true, 0, o.check_every, m.aux));
  // the new slots join the block after the one in flight: `stream` waits for their initialisation
  HIPCHK(hipEventRecord(m.ev_aux, m.aux));
  HIPCHK(hipStreamWaitEvent(m.stream, m.ev_aux, 0));
  m.act.insert(m.act.end(), fresh.begin(), fresh.end());   // (d_slots follows at the next launch_block)
  m.sub_pending[sk] = true;
  return NEP_OK;
}

// The launches of one block (iterations 0 .. ce-1 on `na` iterating slots, m.d_slots) captured
// once as a HIP graph and cached per na; m.d_slots is read by the kernels at run time, so the
// graph replays for any set of na slots.
hipError_t block_graph(Model &m, int na, hipGraphExec_t *out) {
  const int ce = m.run.check_every;
  if (m.graph_ce != ce) {
    for (hipGraphExec_t &g : m.block_graph)
      if (g) { (void)hipGraphExecDestroy(g); g = nullptr; }
    m.block_graph.assign(m.max_batch + 1, nullptr);
    m.graph_ce = ce;
  }
  if (!m.block_graph[na]) {
    hipError_t e = hipStreamBeginCapture(m.stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return e;
    hipError_t le = hipSuccess;
    for (int it = 0; it < ce && le == hipSuccess; ++it) {
      const bool check = it == 0, first = it == 1;
      const bool plain = !kHalpern || ce < 4 || it == 0 || it == ce - 1;
      le = launch_x_pass(m.v, m.d_slots, na, check, false, first, plain, it, m.stream);
      if (le == hipSuccess) le = launch_node_pass(m.v, m.d_slots, na, check, false, first, plain, it, m.stream);
      if (le == hipSuccess && (m.step2 || check))
        le = launch_scalar_pass(m.v, m.d_slots, na, check, false, first, plain, it, ce, m.stream);
    }
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(m.stream, &graph);
    if (le != hipSuccess) { if (graph) (void)hipGraphDestroy(graph); return le; }
    if (e != hipSuccess) return e;
    hipGraphExec_t exec = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return e;
    m.block_graph[na] = exec;
  }
  *out = m.block_graph[na];
  return hipSuccess;
}

// One block of `ce` iterations on the iterating slots (m.act), enqueued without waiting: it == 0 is
// the certificate iteration (a plain PDHG step whose input dual is the previous block's plain
// output, so it satisfies the row sign constraints and its Lagrangian is a valid bound); restarts
// decided there take effect at it == 1; it == ce - 1 is plain again; the others are reflected
// Halpern steps.  Every 4th block runs eagerly with one steady-state x-pass launch bracketed by HIP
// events on the model's stream (nep_get_stats); the others replay the block's launches as one HIP
// graph (a block is 2-3 launches per iteration: at small sizes the iteration is launch-latency
// bound).  The block ends with an async copy of every slot's Ctrl into pinned host memory.
int launch_block(Model &m) {
  DeviceView &v = m.v;
  const int ce = m.run.check_every;
  const int na = (int)m.act.size();
  const int sample_it = (ce >= 4 && m.blocks % 4 == 0) ? 2 : -1;
  m.blocks += 1;
  // the iterating slots for the kernels (read at run time, so the cached graphs replay for any set):
  // staged through pinned memory, rewritten only here — every earlier upload has completed, since a
  // block is launched only once the previous one was waited for (advance) — so no queued copy reads a
  // host buffer that the caller's next submit may reallocate (round-3 ADVICE)
  std::copy(m.act.begin(), m.act.end(), m.h_act);
  HIPCHK(hipMemcpyAsync(m.d_slots, m.h_act, na * sizeof(int32_t), hipMemcpyHostToDevice, m.stream));
  bool eager = sample_it >= 0 || !m.graphs_ok;
  if (!eager) {
    hipGraphExec_t g = nullptr;
    if (block_graph(m, na, &g) != hipSuccess) {
      (void)hipGetLastError();
      m.graphs_ok = false;   // e.g. a caller's stream that cannot be captured
      eager = true;
    } else {
      HIPCHK(hipGraphLaunch(g, m.stream));
      m.stats.x_pass_launches += ce;
    }
  }
  for (int it = 0; it < ce && eager; ++it) {
    const bool check = it == 0, first = it == 1;
    const bool plain = !kHalpern || ce < 4 || it == 0 || it == ce - 1;
    const bool sample = it == sample_it;
    if (sample) HIPCHK(hipEventRecord(m.ev0, m.stream));
    HIPCHK(launch_x_pass(v, m.d_slots, na, check, false, first, plain, it, m.stream));
    if (sample) HIPCHK(hipEventRecord(m.ev1, m.stream));
    HIPCHK(launch_node_pass(v, m.d_slots, na, check, false, first, plain, it, m.stream));
    if (m.step2 || check) HIPCHK(launch_scalar_pass(v, m.d_slots, na, check, false, first, plain, it, ce, m.stream));
    m.stats.x_pass_launches += 1;
  }
  HIPCHK(hipMemcpyAsync(m.h_ctrl, v.ctrl, sizeof(Ctrl) * m.max_batch, hipMemcpyDeviceToHost, m.stream));
  m.stats.lp_iterations += (int64_t)na * ce;
  m.launched = m.act;
  m.inflight = true;
  m.inflight_sampled = sample_it >= 0;
  return NEP_OK;
}

// Run blocks of `check_every` PDHG iterations on every iterating slot until at least `min_done`
// of them have finished (min_done <= 0: exactly one block).  Finished slots are reported in
// done[0 .. *n_done) with their results.  Blocks are pipelined: once a block's results are read,
// the next block of the still-iterating slots is enqueued BEFORE returning, so the device keeps
// iterating while the caller branches, presolves and submits the next nodes (those join at the
// block after; their initialisation is stream-ordered behind the block in flight).
int advance(Model &m, int min_done, int32_t *n_done, int32_t *done, double *obj, double *pobj, int32_t *status,
            int64_t *iters) {
  *n_done = 0;
  while (true) {
    if (!m.inflight) {
      if (m.act.empty()) break;
      int rc = launch_block(m);
      if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(m.stream));
    m.inflight = false;
    if (m.inflight_sampled) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, m.ev0, m.ev1));
      m.stats.x_pass_ms += ms;
      m.stats.x_pass_sampled += 1;
      m.stats.x_pass_lp_iters += (int64_t)m.launched.size();
    }
    // results of the slots that block iterated (slots submitted meanwhile are not in it)
    std::vector<uint8_t> fin(m.max_batch, 0);
    for (int s : m.launched) {
      const Ctrl &c = m.h_ctrl[s];
      if (c.active) continue;
      fin[s] = 1;
      const int k = (*n_done)++;
      done[k] = s;
      status[k] = c.status;
      iters[k] = c.k;
      pobj[k] = c.pobj;
      obj[k] = c.status == NEP_LP_INFEASIBLE ? INF : (c.status == NEP_LP_OPTIMAL ? c.lagr : c.best_lagr);
      m.busy[s] = 0;
    }
    if (*n_done > 0) {
      std::vector<int32_t> still;
      for (int s : m.act)
        if (!fin[s]) still.push_back(s);
      m.act.swap(still);
    }
    // the next block runs while the caller handles the finished slots — unless more than
    // pipe_max_done slots just finished and the call returns: then the caller's refill joins the
    // very next block instead of the one after (NEP_PIPELINE_MAX_DONE; default: always pipeline)
    const bool returning = min_done <= 0 || *n_done >= min_done;
    if (!m.act.empty() && (!returning || *n_done <= m.pipe_max_done)) {
      int rc = launch_block(m);
      if (rc) return rc;
    }
    if (returning) break;
  }
  return NEP_OK;
}

int solve_batch(Model &m, int B, const int32_t *slots, const double *lbi, const double *ubi, const nep_lp_opts *opts,
                double *obj, double *pobj, int32_t *status, int64_t *iters) {
  auto t0 = std::chrono::steady_clock::now();
  if (B <= 0) return NEP_OK;
  if (B > m.max_batch) return fail(NEP_ERR_ARG, "B > max_batch");
  if (!m.act.empty()) return fail(NEP_ERR_STATE, "streamed LPs are still iterating (nep_lp_advance them first)");
  std::vector<int> where(m.max_batch, -1);
  for (int b = 0; b < B; ++b) {
    if (slots[b] < 0 || slots[b] >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
    if (where[slots[b]] >= 0) return fail(NEP_ERR_ARG, "duplicate slot");
    where[slots[b]] = b;
  }
  int rc = submit(m, B, slots, lbi, ubi, opts, status);
  if (rc) return rc;
  for (int b = 0; b < B; ++b) {
    obj[b] = status[b] == NEP_LP_INFEASIBLE ? INF : -INF;
    pobj[b] = NAN;
    iters[b] = 0;
  }
  std::vector<int32_t> dn(m.max_batch), ds(m.max_batch);
  std::vector<double> dobj(m.max_batch), dpobj(m.max_batch);
  std::vector<int64_t> dit(m.max_batch);
  while (!m.act.empty()) {
    int32_t nd = 0;
    rc = advance(m, INT_MAX, &nd, dn.data(), dobj.data(), dpobj.data(), ds.data(), dit.data());
    if (rc) return rc;
    for (int k = 0; k < nd; ++k) {
      const int b = where[dn[k]];
      status[b] = ds[k];
      obj[b] = dobj[k];
      pobj[b] = dpobj[k];
      iters[b] = dit[k];
    }
  }
  m.stats.solve_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return NEP_OK;
}

// ---------------------------------------------------------------------------------------------
// auxiliary device work on finished slots (nep_aux.hip)
// ---------------------------------------------------------------------------------------------
// The solution of a slot: the certificate's repaired point when its LP was certified (that point
// is the one whose objective and feasibility the certificate proved), else the PDHG iterate.
int solution_z(Model &m, int slot, const double **z) {
  int32_t st = 0;
  HIPCHK(hipMemcpyAsync(&st, &m.v.ctrl[slot].status, sizeof(int32_t), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  *z = (st == NEP_LP_OPTIMAL ? m.v.zr : m.v.zi) + (size_t)slot * m.v.sint;
  return NEP_OK;
}

int ensure_entries(Model &m, int64_t need) {
  if (need <= m.ecap) return NEP_OK;
  int64_t cap = std::max<int64_t>(need, 4096);
  int rc;
  if ((rc = dalloc(m, &m.d_erow, (size_t)cap))) return rc;
  if ((rc = dalloc(m, &m.d_ecol, (size_t)cap))) return rc;
  if ((rc = dalloc(m, &m.d_eval, (size_t)cap))) return rc;
  m.ecap = cap;
  return NEP_OK;
}

// compaction of a [rows][ld] device matrix: entries > thr, in row-major order
template <typename T>
int compact(Model &m, const T *vals, int rows, int cols, int64_t ld, double thr, int round3, int64_t capacity,
            int64_t *n_out, int32_t *orow, int32_t *ocol, double *oval) {
  int rc;
  if (!m.d_cnt) {
    const size_t n = (size_t)std::max(m.R, m.F) + 1;
    if ((rc = dalloc(m, &m.d_cnt, n))) return rc;
    if ((rc = dalloc(m, &m.d_off, n))) return rc;
  }
  hipError_t e;
  if constexpr (sizeof(T) == 4)
    e = launch_compact_f32(vals, rows, cols, ld, thr, round3, m.d_cnt, m.d_off, nullptr, nullptr, nullptr, true, m.aux);
  else
    e = launch_compact_f64(vals, rows, cols, ld, thr, round3, m.d_cnt, m.d_off, nullptr, nullptr, nullptr, true, m.aux);
  HIPCHK(e);
  int32_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, m.d_off + rows, sizeof(int32_t), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  *n_out = total;
  if (capacity < total || total == 0) return NEP_OK;   // size query (or nothing to write)
  if ((rc = ensure_entries(m, total))) return rc;
  if constexpr (sizeof(T) == 4)
    e = launch_compact_f32(vals, rows, cols, ld, thr, round3, m.d_cnt, m.d_off, m.d_erow, m.d_ecol, m.d_eval, false,
                           m.aux);
  else
    e = launch_compact_f64(vals, rows, cols, ld, thr, round3, m.d_cnt, m.d_off, m.d_erow, m.d_ecol, m.d_eval, false,
                           m.aux);
  HIPCHK(e);
  if (orow) HIPCHK(hipMemcpyAsync(orow, m.d_erow, total * sizeof(int32_t), hipMemcpyDeviceToHost, m.aux));
  if (ocol) HIPCHK(hipMemcpyAsync(ocol, m.d_ecol, total * sizeof(int32_t), hipMemcpyDeviceToHost, m.aux));
  if (oval) HIPCHK(hipMemcpyAsync(oval, m.d_eval, total * sizeof(double), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  return NEP_OK;
}

int flows(Model &m, int n, const int32_t *slots, float *out, float *wout = nullptr) {
  if (n <= 0) return NEP_OK;
  if (n > m.max_batch) return fail(NEP_ERR_ARG, "n > max_batch");
  for (int b = 0; b < n; ++b) {
    if (slots[b] < 0 || slots[b] >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
    if (m.busy[slots[b]]) return fail(NEP_ERR_STATE, "slot is still iterating");
  }
  int rc;
  const size_t plane = (size_t)m.max_batch * m.F * m.N;
  if (!m.d_flows && (rc = dalloc(m, &m.d_flows, 2 * plane))) return rc;
  // pinned staging both ways: pageable copies cost ~0.3 ms per call while a block iterates (round-4 B&B
  // profile, tools/probes/bnb_profile.py: 2.5 of 10 s at 64x32)
  if (!m.h_flows) {
    void *h = nullptr;
    if (hipHostMalloc(&h, sizeof(float) * 2 * plane + sizeof(int32_t) * m.max_batch) != hipSuccess)
      return fail(NEP_ERR_NOMEM, "hipHostMalloc (flows)");
    m.h_flows = static_cast<float *>(h);
  }
  int32_t *hs = reinterpret_cast<int32_t *>(m.h_flows + 2 * plane);
  std::memcpy(hs, slots, n * sizeof(int32_t));
  const size_t cnt = (size_t)n * m.F * m.N;
  HIPCHK(hipMemcpyAsync(m.d_new, hs, n * sizeof(int32_t), hipMemcpyHostToDevice, m.aux));
  HIPCHK(launch_node_flows(m.v, m.d_new, n, m.d_flows, wout ? m.d_flows + plane : nullptr, m.aux));
  HIPCHK(hipMemcpyAsync(m.h_flows, m.d_flows, cnt * sizeof(float), hipMemcpyDeviceToHost, m.aux));
  if (wout) HIPCHK(hipMemcpyAsync(m.h_flows + plane, m.d_flows + plane, cnt * sizeof(float), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  std::memcpy(out, m.h_flows, cnt * sizeof(float));
  if (wout) std::memcpy(wout, m.h_flows + plane, cnt * sizeof(float));
  return NEP_OK;
}

int score_check(Model &m, int slot, double *out) {
  int rc;
  const size_t nfj = (size_t)m.F * m.NP, nf = (size_t)m.F * 4, nj = (size_t)m.N * 6;
  if (!m.d_score) {
    if ((rc = dalloc(m, &m.d_score, nfj + nf + nj + 16))) return rc;
    const double *p = nullptr;
    if ((rc = upload(m, &p, m.node_cost))) return rc;
    m.d_node_cost = const_cast<double *>(p);
  }
  double *cpu_fj = m.d_score, *fpart = cpu_fj + nfj, *jpart = fpart + nf, *dout = jpart + nj;
  const double *z = nullptr;
  if ((rc = solution_z(m, slot, &z))) return rc;
  HIPCHK(launch_score_check(m.v, slot, z, cpu_fj, fpart, jpart, m.d_node_cost, m.node_budget, dout, m.aux));
  double raw[16] = {0};
  HIPCHK(hipMemcpyAsync(raw, dout, 10 * sizeof(double), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  // NEP_SC_* layout (include/neptune_lp.h)
  out[0] = raw[0];                                   // network delay  sum W D x
  out[1] = raw[6];                                   // nodes used     #{n != 0}
  out[2] = raw[7];                                   // node cost      sum n * cost
  out[3] = raw[1];                                   // c_x violations
  out[4] = raw[3];                                   // memory violations
  out[5] = raw[2];                                   // handle_all violations (sources)
  out[6] = raw[4];                                   // CPU violations
  out[7] = raw[5];                                   // n_c violations
  out[8] = raw[7] > m.node_budget + 1e-6 ? 1.0 : 0.0;   // budget violated
  out[9] = raw[8];                                   // max |sum_j x - 1| over routing rows
  out[10] = raw[9];                                  // max CPU excess over cores
  return NEP_OK;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

int nep_api_version(void) { return NEP_API_VERSION; }
const char *nep_last_error(void) { return g_err.c_str(); }

// API 9: a descriptor whose arrays are device memory (nep_model_desc.device_inputs), staged to the host: the
// build's aggregation, coefficients, presolve base box and scaling read the O(F N + N^2) instance there
struct HostDesc {
  nep_model_desc d{};
  std::vector<double> delay, workload, cpr, fmem, nmem, ncores, ncost, maxd, old;
};
static int stage_device_desc(const nep_model_desc &in, HostDesc &h) {
  h.d = in;
  h.d.device_inputs = 0;
  const size_t N = (size_t)std::max(0, in.n_nodes), F = (size_t)std::max(0, in.n_functions);
  auto get = [&](const double *src, size_t n, std::vector<double> &dst, const double **out) -> hipError_t {
    if (!src) { *out = nullptr; return hipSuccess; }
    dst.resize(n);
    *out = dst.data();
    return n ? hipMemcpy(dst.data(), src, n * sizeof(double), hipMemcpyDeviceToHost) : hipSuccess;
  };
  hipError_t e = hipSuccess;
  if (e == hipSuccess) e = get(in.delay, N * N, h.delay, &h.d.delay);
  if (e == hipSuccess) e = get(in.workload, F * N, h.workload, &h.d.workload);
  if (e == hipSuccess) e = get(in.core_per_req, F * N, h.cpr, &h.d.core_per_req);
  if (e == hipSuccess) e = get(in.function_memory, F, h.fmem, &h.d.function_memory);
  if (e == hipSuccess) e = get(in.node_memory, N, h.nmem, &h.d.node_memory);
  if (e == hipSuccess) e = get(in.node_cores, N, h.ncores, &h.d.node_cores);
  if (e == hipSuccess) e = get(in.node_cost, N, h.ncost, &h.d.node_cost);
  if (e == hipSuccess) e = get(in.max_delay, F, h.maxd, &h.d.max_delay);
  if (e == hipSuccess) e = get(in.old_allocations, F * N, h.old, &h.d.old_allocations);
  if (e != hipSuccess) return fail(NEP_ERR_ARG, std::string("device_inputs: reading the instance arrays: ") +
                                                    hipGetErrorString(e));
  return NEP_OK;
}

int nep_model_create(const nep_model_desc *desc_in, int32_t max_batch, void *hip_stream, void **out_model) {
  if (!desc_in || !out_model) return fail(NEP_ERR_ARG, "null argument");
  HostDesc staged;
  const nep_model_desc *desc = desc_in;
  if (desc_in->device_inputs) {
    const int rs = stage_device_desc(*desc_in, staged);
    if (rs) return rs;
    desc = &staged.d;
  }
  if (max_batch <= 0) return fail(NEP_ERR_ARG, "max_batch must be positive");
  std::unique_ptr<Model> m(new Model());
  // (NEP_HOST_POWER=1: the host power iteration instead of the device's, for A/B)
  const char *hp = std::getenv("NEP_HOST_POWER");
  const bool host_power = hp && std::atoi(hp) != 0;
  int rc = build(*m, *desc, host_power);
  if (rc == NEP_OK) presolve_setup(*m);
  if (rc) return rc;
  rc = setup_device(*m, max_batch, hip_stream);
  if (rc) return rc;
  rc = setup_dense(*m, *desc);
  if (rc) return rc;
  if (!host_power && (rc = power_device(*m))) return rc;
  if (const char *e = std::getenv("NEP_ETA_SCALE")) m->eta *= std::atof(e);   // (probe: tools/probes/root_chaos_probe.py)
  if (const char *e = std::getenv("NEP_HOST_PROFILE")) m->prof = e[0] == '1';
  *out_model = m.release();
  return NEP_OK;
}

void nep_model_destroy(void *model) {
  Model *m = static_cast<Model *>(model);
  if (m && m->prof)
    std::fprintf(stderr, "[nep_lp profile] %dx%d%s | submit calls %lld lps %lld presolve %.3fs staging+launch %.3fs | "
                 "advance calls %lld %.3fs\n", m->N, m->F, m->fac ? " fac" : "", (long long)m->pr_calls,
                 (long long)m->pr_lps, m->pr_pre, m->pr_stage, (long long)m->pr_adv_calls, m->pr_adv);
  delete m;
}

int nep_model_get_info(void *model, nep_model_info *info) {
  if (!model || !info) return fail(NEP_ERR_ARG, "null argument");
  const Model &m = *static_cast<Model *>(model);
  info->n_int = m.il.n_int;
  info->n_rows = m.R;
  info->n_tiles = m.F;
  info->max_batch = m.max_batch;
  info->x_entries = (int64_t)m.R * m.N;
  // B_iter = 4 (2P + 2FN + 2N + 2m), P = x entries iterated, m = dual rows
  // (facility relaxation: the x <= c rows are dualised rows too, one per routing entry: m += R N)
  info->bytes_per_iter = 4 * (2 * (int64_t)m.R * m.N + 2 * (int64_t)m.F * m.N + 2 * (int64_t)m.N +
                              2 * ((int64_t)m.dl.n_dual + (m.fac ? (int64_t)m.R * m.N : 0)));
  info->step_size = m.eta;
  info->primal_weight0 = m.omega0;
  return NEP_OK;
}

int nep_lp_solve_batch(void *model, int32_t B, const int32_t *slots, const double *lb_int, const double *ub_int,
                       const nep_lp_opts *opts, double *obj, double *primal_obj, int32_t *status, int64_t *iters) {
  if (!model || !slots || !obj || !primal_obj || !status || !iters) return fail(NEP_ERR_ARG, "null argument");
  return solve_batch(*static_cast<Model *>(model), B, slots, lb_int, ub_int, opts, obj, primal_obj, status, iters);
}

int nep_lp_submit(void *model, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                  const nep_lp_opts *opts, int32_t *status) {
  if (!model || (n > 0 && (!slots || !status))) return fail(NEP_ERR_ARG, "null argument");
  return submit(*static_cast<Model *>(model), n, slots, lb_int, ub_int, opts, status);
}

int nep_lp_submit_ex(void *model, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                     const nep_lp_opts *opts, const int64_t *max_iters, const double *bound_res, int32_t *status) {
  if (!model || (n > 0 && (!slots || !status))) return fail(NEP_ERR_ARG, "null argument");
  return submit(*static_cast<Model *>(model), n, slots, lb_int, ub_int, opts, status, max_iters, bound_res);
}

int nep_lp_advance(void *model, int32_t min_done, int32_t *n_done, int32_t *done_slots, double *obj,
                   double *primal_obj, int32_t *status, int64_t *iters) {
  if (!model || !n_done || !done_slots || !obj || !primal_obj || !status || !iters)
    return fail(NEP_ERR_ARG, "null argument");
  auto t0 = std::chrono::steady_clock::now();
  Model &m = *static_cast<Model *>(model);
  const int rc = advance(m, min_done, n_done, done_slots, obj, primal_obj, status, iters);
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  m.stats.solve_ms += 1e3 * dt;
  if (m.prof) { m.pr_adv += dt; ++m.pr_adv_calls; }
  return rc;
}

int nep_lp_active(void *model) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  return (int)static_cast<Model *>(model)->act.size();
}

int nep_lp_get_solutions(void *model, int32_t n, const int32_t *slots, double *z_out) {
  if (!model || (n > 0 && (!slots || !z_out))) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (n <= 0) return NEP_OK;
  if (n > m.max_batch) return fail(NEP_ERR_ARG, "n > max_batch");
  for (int b = 0; b < n; ++b) {
    if (slots[b] < 0 || slots[b] >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
    if (m.busy[slots[b]]) return fail(NEP_ERR_STATE, "slot is still iterating");
  }
  const size_t ni = (size_t)m.il.n_int;
  if (!m.h_sols) {
    void *hp = nullptr;
    if (hipHostMalloc(&hp, sizeof(double) * m.max_batch * (ni + 1)) != hipSuccess)
      return fail(NEP_ERR_NOMEM, "hipHostMalloc (solutions)");
    m.h_sols = static_cast<double *>(hp);
  }
  int rc;
  if (!m.d_sols && (rc = dalloc(m, &m.d_sols, (size_t)m.max_batch * ni))) return rc;
  // (the certified point for a certified LP, else the iterate — solution_z's choice, made on the device)
  int32_t *hs = reinterpret_cast<int32_t *>(m.h_sols + (size_t)m.max_batch * ni);
  std::memcpy(hs, slots, n * sizeof(int32_t));
  HIPCHK(hipMemcpyAsync(m.d_new, hs, n * sizeof(int32_t), hipMemcpyHostToDevice, m.aux));
  HIPCHK(launch_gather_solutions(m.v, m.d_new, n, (int)ni, m.d_sols, m.aux));
  HIPCHK(hipMemcpyAsync(m.h_sols, m.d_sols, (size_t)n * ni * sizeof(double), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  std::memcpy(z_out, m.h_sols, sizeof(double) * n * ni);
  return NEP_OK;
}

int nep_lp_get_flows_solutions(void *model, int32_t n, const int32_t *slots, float *flows_out, double *z_out) {
  if (!model || (n > 0 && (!slots || !flows_out || !z_out))) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (n <= 0) return NEP_OK;
  if (n > m.max_batch) return fail(NEP_ERR_ARG, "n > max_batch");
  for (int b = 0; b < n; ++b) {
    if (slots[b] < 0 || slots[b] >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
    if (m.busy[slots[b]]) return fail(NEP_ERR_STATE, "slot is still iterating");
  }
  const size_t ni = (size_t)m.il.n_int, plane = (size_t)m.max_batch * m.F * m.N;
  int rc;
  if (!m.d_flows && (rc = dalloc(m, &m.d_flows, 2 * plane))) return rc;
  if (!m.d_sols && (rc = dalloc(m, &m.d_sols, (size_t)m.max_batch * ni))) return rc;
  if (!m.h_flows) {
    void *h = nullptr;
    if (hipHostMalloc(&h, sizeof(float) * 2 * plane + sizeof(int32_t) * m.max_batch) != hipSuccess)
      return fail(NEP_ERR_NOMEM, "hipHostMalloc (flows)");
    m.h_flows = static_cast<float *>(h);
  }
  if (!m.h_sols) {
    void *hp = nullptr;
    if (hipHostMalloc(&hp, sizeof(double) * m.max_batch * (ni + 1)) != hipSuccess)
      return fail(NEP_ERR_NOMEM, "hipHostMalloc (solutions)");
    m.h_sols = static_cast<double *>(hp);
  }
  // nep_lp_get_flows + nep_lp_get_solutions with one slot list, both gathers and one wait
  int32_t *hs = reinterpret_cast<int32_t *>(m.h_flows + 2 * plane);
  std::memcpy(hs, slots, n * sizeof(int32_t));
  const size_t cnt = (size_t)n * m.F * m.N;
  HIPCHK(hipMemcpyAsync(m.d_new, hs, n * sizeof(int32_t), hipMemcpyHostToDevice, m.aux));
  HIPCHK(launch_node_flows(m.v, m.d_new, n, m.d_flows, nullptr, m.aux));
  HIPCHK(launch_gather_solutions(m.v, m.d_new, n, (int)ni, m.d_sols, m.aux));
  HIPCHK(hipMemcpyAsync(m.h_flows, m.d_flows, cnt * sizeof(float), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipMemcpyAsync(m.h_sols, m.d_sols, (size_t)n * ni * sizeof(double), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  std::memcpy(flows_out, m.h_flows, cnt * sizeof(float));
  std::memcpy(z_out, m.h_sols, sizeof(double) * n * ni);
  return NEP_OK;
}

int nep_lp_get_solution(void *model, int32_t slot, double *z_int, float *x_dense) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (m.busy[slot]) return fail(NEP_ERR_STATE, "slot is still iterating");
  if (z_int) {
    const double *z = nullptr;
    int rc = solution_z(m, slot, &z);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(z_int, z, m.il.n_int * sizeof(double), hipMemcpyDeviceToHost, m.aux));
  }
  if (x_dense) {
    std::vector<float> xb((size_t)m.R * m.NP);
    HIPCHK(hipMemcpyAsync(xb.data(), m.v.x + (size_t)slot * m.v.sx, xb.size() * sizeof(float), hipMemcpyDeviceToHost,
                          m.aux));
    HIPCHK(hipStreamSynchronize(m.aux));
    const int N = m.N, F = m.F;
    for (int r = 0; r < m.R; ++r) {
      const int f = m.row_f[r], src = m.row_src[r];
      const float *xr = &xb[(size_t)r * m.NP];
      for (int i = 0; i < N; ++i) {
        const bool member = src >= 0 ? (i == src) : (m.W[(size_t)f * N + i] == 0.0);
        if (!member) continue;
        std::memcpy(&x_dense[((size_t)i * F + f) * N], xr, N * sizeof(float));   // [i][f][j]
      }
    }
  }
  HIPCHK(hipStreamSynchronize(m.aux));
  return NEP_OK;
}

int nep_lp_get_rows(void *model, int32_t slot, float *xbar, int32_t *row_f, int32_t *row_src) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (xbar && m.busy[slot]) return fail(NEP_ERR_STATE, "slot is still iterating");
  if (xbar) {
    HIPCHK(hipMemcpy2DAsync(xbar, m.N * sizeof(float), m.v.x + (size_t)slot * m.v.sx, m.NP * sizeof(float),
                            m.N * sizeof(float), m.R, hipMemcpyDeviceToHost, m.aux));
    HIPCHK(hipStreamSynchronize(m.aux));
  }
  if (row_f) std::memcpy(row_f, m.row_f.data(), m.R * sizeof(int32_t));
  if (row_src) std::memcpy(row_src, m.row_src.data(), m.R * sizeof(int32_t));
  return NEP_OK;
}

static_assert(sizeof(Ctrl) % 4 == 0, "copy_segments copies 4-byte words");

int nep_lp_copy_state(void *model, int32_t src, int32_t dst) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (src < 0 || dst < 0 || src >= m.max_batch || dst >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (m.busy[dst]) return fail(NEP_ERR_STATE, "destination slot is still iterating");
  // (the copy runs on the aux stream, not ordered after the block in flight: an iterating source would
  // be read while the block rewrites it)
  if (m.busy[src]) return fail(NEP_ERR_STATE, "source slot is still iterating");
  if (src == dst) return NEP_OK;
  const DeviceView &v = m.v;
  // every per-slot array of the iterate, in one launch (copy_segments)
  SlotCopy c{};
  auto seg = [&](auto *base, int64_t stride) {
    c.src[c.n] = reinterpret_cast<const char *>(base + src * stride);
    c.dst[c.n] = reinterpret_cast<char *>(base + dst * stride);
    c.bytes[c.n] = stride * (int64_t)sizeof(*base);
    ++c.n;
  };
  seg(v.x, v.sx);
  seg(v.theta, (int64_t)m.R);
  seg(v.zi, v.sint);
  seg(v.y, v.sdual);
  seg(v.kty, v.skty);
  // the certificate's repaired point travels with the status it belongs to: solution_z() of a copied
  // certified slot returns the source's repaired point, not the destination's stale one
  seg(v.zr, v.sint);
  seg(v.rpart, v.srpart);
  seg(v.ctrl, (int64_t)1);
  if (m.fac) {   // the x <= c duals and their per-(f, j) sums travel with the state
    seg(v.lam, v.sx);
    seg(v.lsum, v.slsum);
  }
  HIPCHK(launch_copy_segments(c, m.aux));
  // no host wait: every later use of src / dst is ordered behind these copies — host reads and submits run
  // on `aux`, and a slot iterates on `stream` only after its submit's initialisation (ev_aux)
  return NEP_OK;
}

int nep_lp_copy_states(void *model, int32_t n, const int32_t *src, const int32_t *dst) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  if (n < 0 || (n > 0 && (!src || !dst))) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  for (int k = 0; k < n; ++k) {
    if (src[k] < 0 || dst[k] < 0 || src[k] >= m.max_batch || dst[k] >= m.max_batch)
      return fail(NEP_ERR_ARG, "slot out of range");
    if (m.busy[dst[k]]) return fail(NEP_ERR_STATE, "destination slot is still iterating");
    if (m.busy[src[k]]) return fail(NEP_ERR_STATE, "source slot is still iterating");
  }
  const DeviceView &v = m.v;
  SlotCopyN c{};
  auto seg = [&](auto *base, int64_t stride) {
    c.base[c.nseg] = reinterpret_cast<char *>(base);
    c.stride[c.nseg] = stride * (int64_t)sizeof(*base);
    ++c.nseg;
  };
  // the arrays nep_lp_copy_state copies
  seg(v.x, v.sx);
  seg(v.theta, (int64_t)m.R);
  seg(v.zi, v.sint);
  seg(v.y, v.sdual);
  seg(v.kty, v.skty);
  seg(v.zr, v.sint);
  seg(v.rpart, v.srpart);
  seg(v.ctrl, (int64_t)1);
  if (m.fac) {
    seg(v.lam, v.sx);
    seg(v.lsum, v.slsum);
  }
  // the same result as n nep_lp_copy_state calls in order: a launch takes pairs while none of them reads or writes
  // a slot an earlier pair of the launch writes, or writes a slot an earlier pair reads
  std::vector<int32_t> rd, wr;
  auto flush = [&]() -> int {
    if (c.npairs) HIPCHK(launch_copy_slots(c, m.aux));
    c.npairs = 0;
    rd.clear();
    wr.clear();
    return NEP_OK;
  };
  auto has = [](const std::vector<int32_t> &a, int32_t x) { return std::find(a.begin(), a.end(), x) != a.end(); };
  for (int k = 0; k < n; ++k) {
    if (src[k] == dst[k]) continue;
    if (c.npairs == SlotCopyN::kPairs || has(wr, src[k]) || has(wr, dst[k]) || has(rd, dst[k])) {
      const int rc = flush();
      if (rc) return rc;
    }
    c.src[c.npairs] = src[k];
    c.dst[c.npairs] = dst[k];
    ++c.npairs;
    rd.push_back(src[k]);
    wr.push_back(dst[k]);
  }
  // (no host wait, as nep_lp_copy_state)
  return flush();
}

int nep_lp_copy_routing(void *dst_model, int32_t dst_slot, void *src_model, int32_t src_slot) {
  if (!dst_model || !src_model) return fail(NEP_ERR_ARG, "null model");
  Model &d = *static_cast<Model *>(dst_model);
  Model &s = *static_cast<Model *>(src_model);
  if (dst_slot < 0 || dst_slot >= d.max_batch || src_slot < 0 || src_slot >= s.max_batch)
    return fail(NEP_ERR_ARG, "slot out of range");
  if (d.busy[dst_slot]) return fail(NEP_ERR_STATE, "destination slot is still iterating");
  if (s.busy[src_slot]) return fail(NEP_ERR_STATE, "source slot is still iterating");
  if (d.R != s.R || d.N != s.N || d.NP != s.NP || d.F != s.F || d.row_f != s.row_f || d.row_src != s.row_src)
    return fail(NEP_ERR_ARG, "the two models' routing rows differ");
  if (&d == &s && dst_slot == src_slot) return NEP_OK;
  // the source's own queued work on its slot first (its aux stream); then the copies on the destination's
  // aux stream, waited for: the source model may rewrite its slot on its own streams right after this call
  HIPCHK(hipStreamSynchronize(s.aux));
  HIPCHK(hipMemcpyAsync(d.v.x + dst_slot * d.v.sx, s.v.x + src_slot * s.v.sx, d.v.sx * sizeof(float),
                        hipMemcpyDeviceToDevice, d.aux));
  HIPCHK(hipMemcpyAsync(d.v.theta + dst_slot * d.R, s.v.theta + src_slot * s.R, d.R * sizeof(float),
                        hipMemcpyDeviceToDevice, d.aux));
  HIPCHK(hipStreamSynchronize(d.aux));
  return NEP_OK;
}

int nep_lp_set_params(void *model, double tol, double cutoff) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (tol > 0) m.run.tol = tol;
  m.run.cutoff = cutoff;
  HIPCHK(set_prm(m, m.run.tol, m.run.cutoff, m.run.gap_tol));
  HIPCHK(hipStreamSynchronize(m.aux));
  return NEP_OK;
}

int nep_lp_set_reference_weight(void *model, double omega_ref) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  if (!(omega_ref >= 0.0) || !std::isfinite(omega_ref)) return fail(NEP_ERR_ARG, "omega_ref must be finite and >= 0");
  static_cast<Model *>(model)->omega_ref = omega_ref;
  return NEP_OK;
}

int nep_lp_get_flows(void *model, int32_t n, const int32_t *slots, float *flows_out) {
  if (!model || (n > 0 && (!slots || !flows_out))) return fail(NEP_ERR_ARG, "null argument");
  return flows(*static_cast<Model *>(model), n, slots, flows_out);
}

int nep_lp_get_flows_split(void *model, int32_t n, const int32_t *slots, float *flows_out, float *wflows_out) {
  if (!model || (n > 0 && (!slots || !flows_out || !wflows_out))) return fail(NEP_ERR_ARG, "null argument");
  return flows(*static_cast<Model *>(model), n, slots, flows_out, wflows_out);
}

int nep_lp_routing_entries(void *model, int32_t slot, double threshold, int32_t round3, int64_t capacity,
                           int64_t *n_entries, int32_t *row, int32_t *dst, double *val) {
  if (!model || !n_entries) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (m.busy[slot]) return fail(NEP_ERR_STATE, "slot is still iterating");
  return compact<float>(m, m.v.x + (size_t)slot * m.v.sx, m.R, m.N, m.NP, threshold, round3, capacity, n_entries, row,
                        dst, val);
}

int nep_lp_allocation_entries(void *model, int32_t slot, double threshold, int64_t capacity, int64_t *n_entries,
                              int32_t *fn, int32_t *dst) {
  if (!model || !n_entries) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (m.busy[slot]) return fail(NEP_ERR_STATE, "slot is still iterating");
  const double *z = nullptr;
  int rc = solution_z(m, slot, &z);
  if (rc) return rc;
  return compact<double>(m, z + m.il.oc, m.F, m.N, m.N, threshold, 0, capacity, n_entries, fn, dst, nullptr);
}

int nep_lp_score_check(void *model, int32_t slot, double *out) {
  if (!model || !out) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (m.busy[slot]) return fail(NEP_ERR_STATE, "slot is still iterating");
  return score_check(m, slot, out);
}

int nep_lp_get_diag(void *model, int32_t slot, double *out16) {
  if (!model || !out16) return fail(NEP_ERR_ARG, "null argument");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  Ctrl c;
  // read on the auxiliary stream: submits and state copies are enqueued there without a host
  // wait, so a blocking copy on the null stream could see a slot's Ctrl before they ran
  HIPCHK(hipMemcpyAsync(&c, m.v.ctrl + slot, sizeof(Ctrl), hipMemcpyDeviceToHost, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  const double vals[16] = {c.pobj, c.lagr, c.best_lagr, c.pres, c.gap, c.omega, c.tau, c.sigma, c.eta,
                           (double)c.k, (double)c.k_since_restart, (double)c.status, (double)c.active,
                           c.last_restart_fpr, c.prev_fpr, m.sigma_max};
  std::memcpy(out16, vals, sizeof(vals));
  return NEP_OK;
}

int nep_debug_state(void *model, int32_t slot, double *y, double *kz, float *kty, double *lb, double *ub) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  const DeviceView &v = m.v;
  // (stream-ordered behind the submits / copies on the auxiliary stream, as nep_lp_get_diag)
  const hipMemcpyKind d2h = hipMemcpyDeviceToHost;
  if (y) HIPCHK(hipMemcpyAsync(y, v.y + slot * v.sdual, v.sdual * sizeof(double), d2h, m.aux));
  if (kz) HIPCHK(hipMemcpyAsync(kz, v.kz + slot * v.sdual, v.sdual * sizeof(double), d2h, m.aux));
  if (kty) HIPCHK(hipMemcpyAsync(kty, v.kty + slot * v.skty, v.skty * sizeof(float), d2h, m.aux));
  if (lb) HIPCHK(hipMemcpyAsync(lb, v.lb + slot * v.sint, v.sint * sizeof(double), d2h, m.aux));
  if (ub) HIPCHK(hipMemcpyAsync(ub, v.ub + slot * v.sint, v.sint * sizeof(double), d2h, m.aux));
  HIPCHK(hipStreamSynchronize(m.aux));
  return NEP_OK;
}

int nep_debug_sparse_rows(void *model, int32_t slot, int32_t *anchor_cnt, float *lambda_nnz) {
  if (!model) return fail(NEP_ERR_ARG, "null model");
  Model &m = *static_cast<Model *>(model);
  if (slot < 0 || slot >= m.max_batch) return fail(NEP_ERR_ARG, "slot out of range");
  if (lambda_nnz && !m.fac) return fail(NEP_ERR_ARG, "not a facility-relaxation model");
  const DeviceView &v = m.v;
  const hipMemcpyKind d2h = hipMemcpyDeviceToHost;
  if (anchor_cnt) HIPCHK(hipMemcpyAsync(anchor_cnt, v.acnt + (int64_t)slot * m.R, m.R * sizeof(int32_t), d2h, m.aux));
  std::vector<float> lam;
  if (lambda_nnz) {
    lam.resize((size_t)v.sx);
    HIPCHK(hipMemcpyAsync(lam.data(), v.lam + slot * v.sx, lam.size() * sizeof(float), d2h, m.aux));
  }
  HIPCHK(hipStreamSynchronize(m.aux));
  for (int r = 0; lambda_nnz && r < m.R; ++r) {   // (nonzeros of each row of the x <= c duals, host count)
    int c = 0;
    for (int j = 0; j < m.N; ++j) c += lam[(size_t)r * m.NP + j] != 0.f;
    lambda_nnz[r] = (float)c;
  }
  return NEP_OK;
}

int nep_debug_build(const nep_model_desc *desc, double *eta, double *rho, double *gam, double *rownorm, int32_t *dims) {
  if (!desc) return fail(NEP_ERR_ARG, "null argument");
  if (desc->device_inputs) return fail(NEP_ERR_ARG, "nep_debug_build takes host arrays (device_inputs = 0)");
  Model m;
  int rc = build(m, *desc);
  if (rc) return rc;
  if (eta) *eta = m.eta;
  if (rho) std::memcpy(rho, m.rho.data(), m.rho.size() * sizeof(double));
  if (gam) std::memcpy(gam, m.gam.data(), m.gam.size() * sizeof(double));
  if (rownorm) std::memcpy(rownorm, m.rownorm.data(), m.rownorm.size() * sizeof(double));
  if (dims) {
    dims[0] = m.R; dims[1] = m.F; dims[2] = m.il.n_int; dims[3] = m.dl.n_dual;
  }
  return NEP_OK;
}

int nep_get_stats(void *model, nep_stats *stats) {
  if (!model || !stats) return fail(NEP_ERR_ARG, "null argument");
  *stats = static_cast<Model *>(model)->stats;
  return NEP_OK;
}

void nep_reset_stats(void *model) {
  if (model) static_cast<Model *>(model)->stats = nep_stats{};
}

}  // extern "C"

int nep_debug_presolve(const nep_model_desc *desc, int32_t n, const double *lbi, const double *ubi, int32_t *ok_full,
                       int32_t *ok_node, double *box_full, double *box_node) {
  if (!desc || n < 0 || !ok_full || !ok_node) return fail(NEP_ERR_ARG, "null argument");
  if (desc->device_inputs) return fail(NEP_ERR_ARG, "nep_debug_presolve takes host arrays (device_inputs = 0)");
  Model m;
  int rc = build(m, *desc);
  if (rc) return rc;
  presolve_setup(m);
  const size_t ni = (size_t)m.il.n_int;
  std::vector<double> lb, ub;
  std::vector<uint8_t> mask;
  std::vector<NodeBox> box;
  presolve_batch(m, n, lbi, ubi, box);
  for (int b = 0; b < n; ++b)
    if (box[b].bad)
      return fail(NEP_ERR_ARG, "step-2 node box " + std::to_string(b) +
                               ": moved_from / moved_to bounds must be integral (binary variables; NEP_STEP2_FULL=1 "
                               "iterates the full disruption rows)");   // (the submit path: in parallel for large models)
  for (int b = 0; b < n; ++b) {
    const double *l = lbi ? lbi + b * ni : nullptr, *u = ubi ? ubi + b * ni : nullptr;
    ok_full[b] = presolve_full(m, l, u, lb, ub, mask) ? 1 : 0;
    if (box_full) {
      std::memcpy(box_full + 2 * b * ni, lb.data(), ni * sizeof(double));
      std::memcpy(box_full + (2 * b + 1) * ni, ub.data(), ni * sizeof(double));
    }
    const NodeBox &nb = box[b];
    const PresolveScratch &sc = m.psc[nb.t];
    ok_node[b] = nb.ok ? 1 : 0;
    if (box_node) {
      double *bl = box_node + 2 * b * ni, *bu = box_node + (2 * b + 1) * ni;
      std::memcpy(bl, m.base_lb.data(), ni * sizeof(double));
      std::memcpy(bu, m.base_ub.data(), ni * sizeof(double));
      for (size_t t = nb.off; t < nb.off + nb.cnt; ++t) {
        bl[sc.ci[t]] = sc.cl[t];
        bu[sc.ci[t]] = sc.cu[t];
      }
    }
  }
  return NEP_OK;
}
