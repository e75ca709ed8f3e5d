// nep_bnb.cpp — the branch-and-bound's tree search, native (include/neptune_lp.h nep_bnb_*).
//
// The streaming best-first search of core/engine/bnb.py (BranchAndBound.solve, single rank) as a C++ client of
// the engine's C ABI: the open-node heap, the rounding-leaf and retry queues, node selection, the warm-start
// source of every submit (parent slot / root state), the per-engine slot free lists, each finished LP's
// processing (prune, incumbent, retry, branching variable, rounding leaves, children) and the submit of the
// next nodes all run here, one call per search (nep_bnb_run returns only for the events the Python caller
// handles: the root's primal heuristic, the end).  It replaces, per finished node LP, ~30 Python / numpy calls
// (the host share of the 64x32 search, DESIGN.md §7 "Native tree search").  Decision order and tie-breaks are
// bnb.py's, so the two searches visit the same tree (tests/test_gpu_bnb_native.py compares them).
//
// API 12: the models are reached through a call table (nep_bnb_engine: nep_lp_* on an engine handle, or a
// caller's own — the CPU suite drives the tree over HiGHS node LPs, tests/test_bnb_native_cpu.py), and the
// sharded search runs here too: with world > 1 the tree stops once per loop with NEP_BNB_SYNC for the caller's
// one collective (incumbent MIN, stop OR, open count SUM; core/engine/comm.py agree), deals the frontier at
// world x batch open nodes (the same canonical order and crc32 as bnb.py) and exports / imports open nodes for
// the caller's rebalance.
//
// Reference: SCIP's tree search inside pywraplp Solver.Solve() (core/solvers/solver.py:35-40).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <limits>
#include <memory>
#include <queue>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../include/neptune_lp.h"

namespace nep {
int set_error(int code, const char *msg);   // nep_host.cpp: nep_last_error's thread-local message
}

namespace {

int bad(int code, const char *msg) { return nep::set_error(code, msg); }

constexpr double INF = std::numeric_limits<double>::infinity();
enum Kind { NODE = 0, LEAF = 1, RETRY = 2, REFROOT = 3, STRONG = 4 };   // STRONG: a strong-branching probe LP
// lp status columns of nep_bnb_stats.lp_status: certified, bound, limit, infeasible, cutoff, numerical, presolve
int status_col(int st) {
  switch (st) {
    case NEP_LP_OPTIMAL: return 0;
    case NEP_LP_BOUND: return 1;
    case NEP_LP_ITERATION_LIMIT: return 2;
    case NEP_LP_INFEASIBLE: return 3;
    case NEP_LP_CUTOFF: return 4;
    default: return 5;
  }
}

struct Engine;
struct Parent {
  Engine *eng = nullptr;
  int slot = -1;
  int64_t gen = -1;
};
struct SbWait;

struct Node {
  double bound;
  std::vector<int32_t> idx;
  std::vector<double> val;
  int kind;
  Parent parent;
  int depth;
  // the branching that made this node (pseudo-costs): variable, direction (1 = up), the parent LP's distance to
  // the fixed value, the parent's bound
  int bvar = -1, bdir = 0;
  double bfrac = 0.0, pbound = -std::numeric_limits<double>::infinity();
  std::shared_ptr<SbWait> sb;   // STRONG: the branching node its probe belongs to, candidate sb_i
  int sb_i = -1;
};
using NodeP = std::shared_ptr<Node>;

// a branching node waiting for its strong-branching probes (p.branching == 2): candidate variables, their LP values,
// and per direction the probe's bound (NaN pending, +inf infeasible / cut off) and its finished slot (the child's
// warm-start state: the probe ran on the child's own box)
struct SbWait {
  NodeP node;
  Parent at;
  double bound = 0.0;
  std::vector<int> cand;
  std::vector<double> zc, est[2];
  std::vector<char> probed;
  std::vector<double> res[2];
  std::vector<Parent> src[2];
  int pending = 0;
};

struct Engine {
  nep_bnb_engine ops{};         // the model's calls (ops.ctx: the engine handle for nep_lp_*)
  int n_int = 0;                // this model's integer vector length (its boxes, solutions)
  int max_batch = 0, reserved = 0, root_slot = -1, inc_slot = -1;
  std::vector<int64_t> gen;
  std::deque<int> free;
  bool root_ready = false, root_state = false;
  int inflight = 0;
  std::vector<NodeP> running;   // slot -> node in flight
};

struct HeapItem {
  double bound;
  int negdepth;
  int64_t seq;
  NodeP node;
  bool operator>(const HeapItem &o) const {   // min-heap on (bound, -depth, seq), as bnb.py's heapq tuples
    if (bound != o.bound) return bound > o.bound;
    if (negdepth != o.negdepth) return negdepth > o.negdepth;
    return seq > o.seq;
  }
};

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// zlib's crc32 (poly 0xEDB88320), chained like zlib.crc32(data, crc): the frontier hash of bnb.py
uint32_t crc32_update(uint32_t crc, const void *data, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  const unsigned char *p = static_cast<const unsigned char *>(data);
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xFFu] ^ (crc >> 8);
  return ~crc;
}

// the nep_lp_* calls of an engine model as a call table (ctx = the model handle)
int op_submit(void *c, int32_t n, const int32_t *sl, const double *lb, const double *ub, const nep_lp_opts *o,
              int32_t *st) { return nep_lp_submit(c, n, sl, lb, ub, o, st); }
int op_submit_ex(void *c, int32_t n, const int32_t *sl, const double *lb, const double *ub, const nep_lp_opts *o,
                 const int64_t *mi, const double *br, int32_t *st) {
  return nep_lp_submit_ex(c, n, sl, lb, ub, o, mi, br, st);
}
int op_advance(void *c, int32_t md, int32_t *nd, int32_t *sl, double *ob, double *po, int32_t *st, int64_t *it) {
  return nep_lp_advance(c, md, nd, sl, ob, po, st, it);
}
int op_active(void *c) { return nep_lp_active(c); }
int op_copy(void *c, int32_t a, int32_t b) { return nep_lp_copy_state(c, a, b); }
int op_copies(void *c, int32_t n, const int32_t *a, const int32_t *b) { return nep_lp_copy_states(c, n, a, b); }
int op_flows_sols(void *c, int32_t n, const int32_t *sl, float *f, double *z) {
  return nep_lp_get_flows_solutions(c, n, sl, f, z);
}
int op_params(void *c, double tol, double cut) { return nep_lp_set_params(c, tol, cut); }
int op_flows(void *c, int32_t n, const int32_t *sl, float *f) { return nep_lp_get_flows(c, n, sl, f); }
int op_sols(void *c, int32_t n, const int32_t *sl, double *z) { return nep_lp_get_solutions(c, n, sl, z); }
int op_diag(void *c, int32_t s, double *o) { return nep_lp_get_diag(c, s, o); }

int model_ops(void *lp, nep_bnb_engine *out) {
  nep_model_info info{};
  const int rc = nep_model_get_info(lp, &info);
  if (rc) return rc;
  *out = nep_bnb_engine{};
  out->ctx = lp;
  out->n_int = info.n_int;
  out->max_batch = info.max_batch;
  out->submit = op_submit;
  out->advance = op_advance;
  out->active = op_active;
  out->copy_state = op_copy;
  out->set_params = op_params;
  out->get_flows = op_flows;
  out->get_solutions = op_sols;
  out->get_diag = op_diag;
  out->submit_ex = op_submit_ex;
  out->copy_states = op_copies;
  out->get_flows_solutions = op_flows_sols;
  return NEP_OK;
}

}  // namespace

struct NepBnb {
  nep_bnb_params p{};
  Engine L, B;
  bool two = false;
  // NEP_BNB_PROFILE=1: host seconds per section, printed to stderr when the tree is destroyed (dev measurement)
  bool prof = false;
  double pr_round = 0, pr_reads = 0, pr_copies = 0, pr_submit = 0, pr_finish = 0;
  int64_t pr_submit_calls = 0, pr_copy_calls = 0, pr_reads_calls = 0, pr_rounds = 0;
  ~NepBnb() {
    if (prof)
      std::fprintf(stderr,
                   "[nep_bnb profile] lps %lld | submit calls %lld %.3fs, copies calls %lld %.3fs | reads calls %lld "
                   "%.3fs | rounding nodes %lld %.3fs | finish_one %.3fs\n",
                   (long long)st.lps, (long long)pr_submit_calls, pr_submit, (long long)pr_copy_calls, pr_copies,
                   (long long)pr_reads_calls, pr_reads, (long long)pr_rounds, pr_round, pr_finish);
  }
  std::vector<double> fn_mem, node_mem;
  std::priority_queue<HeapItem, std::vector<HeapItem>, std::greater<HeapItem>> heap;
  std::deque<NodeP> pending, retry;
  std::vector<NodeP> seeds;   // seed leaves, queued when the root finishes
  NodeP refroot;
  std::unordered_set<std::string> seen;
  std::vector<int32_t> leaf_idx;   // the variables a rounding leaf fixes (built at the first one)
  std::vector<double> unresolved_bounds;
  std::vector<int64_t> lp_iters;
  int64_t seq = 0;
  double inc = INF;          // this rank's incumbent (its own LP leaves / heuristic points)
  double cut = INF;          // sharded search: the incumbent the ranks agreed on (prunes like inc)
  int inc_source = 0;        // 0 none, 1 an LP leaf (inc_slot / kept slot), 2 external (nep_bnb_set_incumbent)
  int inc_slot = -1;         // slot of the leaf engine holding the incumbent's state
  int keep_slot = -1;        // (warm = 0) a working slot kept for the incumbent
  NodeP inc_node;
  std::vector<double> inc_z;
  nep_bnb_stats st{};
  double t0 = 0.0;
  bool started = false, finished = false, limit_hit = false;
  // the root event (primal heuristic at the root branching node)
  bool root_event_pending = false, root_event_done = false;
  std::vector<double> ev_z;
  std::vector<float> ev_flow;
  NodeP ev_node;
  Parent ev_parent;
  double ev_bound = -INF;
  // step 2 (nep_bnb_set_step2): the closed-form integer bound of NeptuneStep2Base.integer_bound and the
  // incumbent event for its node-relocation neighbours (NeptuneStep2Base.improve, run by the caller)
  bool s2 = false, s2_create = false, inc_events = false;
  double s2_cap = INF;
  std::vector<char> s2_old;   // [F*N] old allocation > 0.5
  struct IncEvent {
    NodeP node;
    Parent at;
    double value;
  };
  std::deque<IncEvent> inc_queue;
  IncEvent cur_inc;
  // sharded search (p.world > 1): one NEP_BNB_SYNC per loop for the caller's collective
  bool split = false;        // the frontier has been dealt (before: every rank runs the same search)
  bool sync_answered = false;
  double sync_out[6] = {0, 0, 0, 0, 0, 0};   // incumbent, stop, open, heap size, split, loops
  double agreed_inc = INF;
  bool agreed_stop = false;
  int64_t agreed_open = 0;
  bool stalled = false;      // nothing could be submitted and nothing was in flight (ends the search)
  // scratch
  std::vector<int32_t> sl, done_slots, sts, cp_src, cp_dst;
  std::vector<double> obj, pobj, lbv, ubv;
  std::vector<int64_t> its;

  int nb() const { return (p.c1 - p.c0) + (p.n0 >= 0 ? p.n1 - p.n0 : 0); }
  double ibound(const std::vector<int32_t> &idx, const std::vector<double> &val) const;
  double gap_abs(double incv) const {
    if (!std::isfinite(incv)) return 0.0;
    double g = p.gap * std::max(1.0, std::fabs(incv));
    if (p.objective_integral) {
      // bound >= inc - unit + delta prunes: no integral point lies strictly between (delta: the fp64 error of a
      // Lagrangian bound of this size, and the reference's eps-scale terms)
      const double u = p.objective_unit > 0 ? p.objective_unit : 1.0;
      g = std::max(g, u * (1.0 - std::min(0.5, 1e-6 + 1e-9 * std::fabs(incv) / u)));
    }
    return g;
  }
  double incv() const { return std::min(inc, cut); }   // the pruning incumbent (the agreed one when sharded)
  bool pruned(double bound) const { return bound >= incv() - gap_abs(incv()); }
  static std::string key_of(const std::vector<double> &val) {
    std::string k((val.size() + 7) / 8, '\0');
    for (size_t i = 0; i < val.size(); ++i)
      if (val[i] > 0.5) k[i / 8] = (char)(k[i / 8] | (0x80 >> (i % 8)));
    return k + std::to_string(val.size());
  }
  void push_heap(const NodeP &n) { heap.push(HeapItem{n->bound, -n->depth, seq++, n}); }
  Engine *engines[2] = {nullptr, nullptr};
  int n_engines() const { return two ? 2 : 1; }

  int set_cutoffs() {
    for (int e = 0; e < n_engines(); ++e) {
      const nep_bnb_engine &o = engines[e]->ops;
      const int rc = o.set_params(o.ctx, p.tol, std::min(incv(), p.upper_bound));
      if (rc) return rc;
    }
    return NEP_OK;
  }
  void deal_frontier();
  int export_nodes(int k, int32_t cap, int32_t *lens, double *meta, int32_t *idx, double *val);

  int submit(std::vector<std::pair<Engine *, std::pair<int, NodeP>>> &items);
  int finish_block(Engine &eng, int nd);
  int finish_one(Engine &eng, int slot, const NodeP &node, int status, double o, double po, int64_t iters,
                 const float *flow, const double *z);
  void round_all(const Node &node, const float *flow, const double *z, double bound, const Parent &me);
  int branch_var(const Node &node, const float *flow, const double *z) const;
  int branch_var_pc(const Node &node, const float *flow, const double *z) const;
  // pseudo-costs (p.branching == 1): per integer variable and direction, the sum / count of the bound gain per unit
  // of fractionality its branchings produced, and the running totals per variable kind (c / n) for the unknown ones
  std::vector<double> pc_sum[2];
  std::vector<int32_t> pc_cnt[2];
  double pck_sum[2][2] = {{0, 0}, {0, 0}};   // [kind: 0 c, 1 n][direction]
  int64_t pck_cnt[2][2] = {{0, 0}, {0, 0}};
  void pc_update(const Node &node, double gain_bound);
  // strong branching (reliability branching: probes only for candidates whose pseudo-costs are unreliable)
  std::deque<NodeP> strong_q;
  int64_t sb_waiting = 0;
  int start_strong(const NodeP &node, const float *flow, const double *z, double bound, const Parent &me);
  void decide_strong(SbWait &w);
  int drain_and_close();
};

namespace {

void init_engine(Engine &e, const nep_bnb_engine &ops, int reserved) {
  e.ops = ops;
  e.n_int = ops.n_int;
  e.max_batch = ops.max_batch;
  e.reserved = ops.max_batch > reserved ? reserved : 0;
  e.root_slot = ops.max_batch - 1;
  e.inc_slot = ops.max_batch - 2;
  e.gen.assign(ops.max_batch, 0);
  e.running.assign(ops.max_batch, nullptr);
  for (int s = 0; s < ops.max_batch - e.reserved; ++s) e.free.push_back(s);
}

bool ops_complete(const nep_bnb_engine &o) {
  return o.submit && o.advance && o.active && o.copy_state && o.set_params && o.get_flows && o.get_solutions &&
         o.get_diag && o.n_int > 0 && o.max_batch > 0;
}

}  // namespace

// one submit per (engine, warm, check_every) group — and per (budget, bound_res) too when the engine has no
// submit_ex (per-LP budgets) — warm-start copies first
int NepBnb::submit(std::vector<std::pair<Engine *, std::pair<int, NodeP>>> &items) {
  struct Group {
    Engine *eng;
    bool warm;
    int64_t budget;
    double bres;
    int ce;
    std::vector<std::pair<int, NodeP>> its;
    std::vector<int64_t> mi;
    std::vector<double> br;
  };
  std::vector<Group> groups;
  std::vector<std::pair<int, int>> copies[2];   // per engine (leaf first): (src, dst)
  const double cutoff = std::min(incv(), p.upper_bound);
  for (auto &it : items) {
    Engine *eng = it.first;
    const int slot = it.second.first;
    const NodeP &node = it.second.second;
    bool warm = false;
    int src = -1;
    if (p.warm && eng->root_ready) {
      src = eng->root_state ? eng->root_slot : -1;
      if (node->parent.eng == eng && node->parent.slot >= 0 && eng->gen[node->parent.slot] == node->parent.gen)
        src = node->parent.slot;
      if (src >= 0) {
        if (src != slot) copies[eng == &L ? 0 : 1].push_back({src, slot});
        warm = true;
      }
    }
    const int64_t budget = (node->kind == RETRY || node->kind == REFROOT || !eng->root_ready)
                               ? p.root_max_iters
                               : (node->kind == NODE ? p.node_max_iters
                                                     : (node->kind == STRONG ? p.strong_iters : p.max_iters));
    const double bres = ((node->kind == NODE || node->kind == STRONG) && (eng->root_ready || two)) ? p.node_bound_res
                                                                                                  : 0.0;
    const int ce = (node->kind == REFROOT || !eng->root_ready) ? p.root_check_every : p.check_every;
    const bool ex = eng->ops.submit_ex != nullptr;
    const int64_t gb = ex ? -1 : budget;
    const double gr = ex ? -1.0 : bres;
    Group *g = nullptr;
    for (auto &gg : groups)
      if (gg.eng == eng && gg.warm == warm && gg.budget == gb && gg.bres == gr && gg.ce == ce) g = &gg;
    if (!g) {
      groups.push_back(Group{eng, warm, gb, gr, ce, {}, {}, {}});
      g = &groups.back();
    }
    g->its.push_back({slot, node});
    g->mi.push_back(budget);
    g->br.push_back(bres);
  }
  // copies: a slot that is both a parent state (source) and a new node's slot (destination) is read before
  // it is overwritten; a cycle falls back to the root's state
  for (int e = 0; e < 2; ++e) {
    Engine *eng = e == 0 ? &L : &B;
    auto &cps = copies[e];
    cp_src.clear();
    cp_dst.clear();
    while (!cps.empty()) {
      size_t k = cps.size();
      for (size_t i = 0; i < cps.size() && k == cps.size(); ++i) {
        bool is_src = false;
        for (auto &c : cps) is_src |= c.first == cps[i].second;
        if (!is_src) k = i;
      }
      if (k == cps.size()) {
        cps[0].first = eng->root_slot;
        continue;
      }
      const auto c = cps[k];
      cps.erase(cps.begin() + k);
      cp_src.push_back(c.first);
      cp_dst.push_back(c.second);
    }
    // in that order: one call (nep_lp_copy_states: as few launches as the overlaps allow), else one per pair
    const double tc = prof ? now_s() : 0.0;
    if (prof && !cp_src.empty()) ++pr_copy_calls;
    if (!cp_src.empty() && eng->ops.copy_states) {
      int rc = eng->ops.copy_states(eng->ops.ctx, (int)cp_src.size(), cp_src.data(), cp_dst.data());
      if (rc) return rc;
    } else {
      for (size_t q = 0; q < cp_src.size(); ++q) {
        int rc = eng->ops.copy_state(eng->ops.ctx, cp_src[q], cp_dst[q]);
        if (rc) return rc;
      }
    }
    if (prof) pr_copies += now_s() - tc;
  }
  for (auto &g : groups) {
    const int n = (int)g.its.size(), ni = g.eng->n_int;
    sl.resize(n);
    lbv.assign((size_t)n * ni, -INF);
    ubv.assign((size_t)n * ni, INF);
    for (int b = 0; b < n; ++b) {
      sl[b] = g.its[b].first;
      const Node &nd = *g.its[b].second;
      for (size_t q = 0; q < nd.idx.size(); ++q) {
        lbv[(size_t)b * ni + nd.idx[q]] = nd.val[q];
        ubv[(size_t)b * ni + nd.idx[q]] = nd.val[q];
      }
    }
    nep_lp_opts o{};
    o.tol = p.tol;
    o.cutoff = std::isfinite(cutoff) ? cutoff : INF;
    o.max_iters = g.mi[0];
    o.check_every = g.ce;
    o.warm_start = g.warm ? 1 : 0;
    o.gap_tol = (two && g.eng == &B) ? p.bound_gap : 0.0;
    o.bound_res = g.br[0];
    sts.assign(n, 0);
    // (a bound-stop entry of 0 means none: nep_lp_submit_ex reads entries <= 0 that way)
    const double ts = prof ? now_s() : 0.0;
    int rc = g.eng->ops.submit_ex
                 ? g.eng->ops.submit_ex(g.eng->ops.ctx, n, sl.data(), lbv.data(), ubv.data(), &o, g.mi.data(),
                                        g.br.data(), sts.data())
                 : g.eng->ops.submit(g.eng->ops.ctx, n, sl.data(), lbv.data(), ubv.data(), &o, sts.data());
    if (prof) { pr_submit += now_s() - ts; ++pr_submit_calls; }
    if (rc) return rc;
    for (int b = 0; b < n; ++b) {
      const int slot = sl[b];
      const NodeP &node = g.its[b].second;
      g.eng->gen[slot] += 1;
      st.lps += 1;
      if (sts[b] == NEP_LP_INFEASIBLE && node->kind == STRONG) {
        st.strong_lps += 1;
        pc_update(*node, incv());
        SbWait &w = *node->sb;
        w.res[node->bdir][node->sb_i] = INF;
        g.eng->free.push_back(slot);
        if (--w.pending == 0) decide_strong(w);
        continue;
      }
      if (sts[b] == NEP_LP_INFEASIBLE) {
        if (p.branching >= 1 && node->kind == NODE) pc_update(*node, incv());
        st.lp_status[6] += 1;
        st.lp_status_kind[node->kind][6] += 1;
        g.eng->free.push_back(slot);
        if (node->kind == REFROOT) g.eng->root_ready = true;   // every leaf is a sub-box of it: no root state
      } else {
        g.eng->running[slot] = node;
        g.eng->inflight += 1;
      }
    }
  }
  return NEP_OK;
}

// one finished child LP: its bound gain over the parent's, per unit of the parent LP's fractionality
void NepBnb::pc_update(const Node &node, double child_bound) {
  if (node.bvar < 0 || !(node.pbound > -INF) || !std::isfinite(child_bound)) return;
  if (pc_sum[0].empty()) {
    for (int d = 0; d < 2; ++d) {
      pc_sum[d].assign(L.n_int, 0.0);
      pc_cnt[d].assign(L.n_int, 0);
    }
  }
  if (node.bvar >= (int)pc_sum[0].size()) return;
  const double g = std::max(0.0, child_bound - node.pbound) / std::max(node.bfrac, 1e-6);
  const int d = node.bdir, k = (p.n0 >= 0 && node.bvar >= p.n0 && node.bvar < p.n1) ? 1 : 0;
  pc_sum[d][node.bvar] += g;
  pc_cnt[d][node.bvar] += 1;
  pck_sum[k][d] += g;
  pck_cnt[k][d] += 1;
}

// pseudo-cost branching (SCIP's default family, here without strong-branching initialisation): among the free c /
// n whose LP value is fractional (and, for c, that carry flow), the largest product score
// max(psi_down z, eps) * max(psi_up (1 - z), eps); a variable never branched takes its kind's average pseudo-cost
// (1 before any).  No fractional candidate: the flow rule below.
// reliability branching: the top strong_cands candidates by pseudo-cost score; those whose pseudo-costs rest on
// fewer than strong_rel observations in either direction get two probe LPs each (STRONG nodes, strong_iters
// iterations, warm from this node's state, on the same model), submitted ahead of every other node; the node
// branches when its probes are back (decide_strong).  Returns 1 when probes were queued, 0 when the pseudo-costs
// decide at once.
int NepBnb::start_strong(const NodeP &node, const float *flow, const double *z, double bound, const Parent &me) {
  const int FN = p.F * p.N;
  std::vector<char> fixed(std::max(p.c1, p.n1) + 1, 0);
  for (int32_t i : node->idx) fixed[i] = 1;
  const double ftol = 1e-4, eps = 1e-6;
  double avg[2][2];
  for (int k = 0; k < 2; ++k)
    for (int d = 0; d < 2; ++d)
      avg[k][d] = pck_cnt[k][d] > 0 ? pck_sum[k][d] / (double)pck_cnt[k][d]
                                    : (pck_cnt[k][1 - d] > 0 ? pck_sum[k][1 - d] / (double)pck_cnt[k][1 - d] : 1.0);
  const bool have = !pc_sum[0].empty();
  struct C { double sc; int v; int rel; double e0, e1; };
  std::vector<C> cs;
  auto consider = [&](int v, int k) {
    const double zf = z[v];
    if (!(zf > ftol && zf < 1.0 - ftol)) return;
    const int n0 = have ? pc_cnt[0][v] : 0, n1 = have ? pc_cnt[1][v] : 0;
    const double p0 = n0 > 0 ? pc_sum[0][v] / n0 : avg[k][0], p1 = n1 > 0 ? pc_sum[1][v] / n1 : avg[k][1];
    const double e0 = p0 * zf, e1 = p1 * (1.0 - zf);
    cs.push_back(C{std::max(e0, eps) * std::max(e1, eps), v, std::min(n0, n1), e0, e1});
  };
  if (p.n0 >= 0)
    for (int v = p.n0; v < p.n1; ++v)
      if (!fixed[v]) consider(v, 1);
  for (int q = 0; q < FN; ++q)
    if (!fixed[p.c0 + q] && (double)flow[q] > p.flow_tol) consider(p.c0 + q, 0);
  if (cs.empty()) return 0;
  std::sort(cs.begin(), cs.end(), [](const C &a, const C &b) { return a.sc != b.sc ? a.sc > b.sc : a.v < b.v; });
  const int K = std::min((int)cs.size(), std::max(1, p.strong_cands));
  int unrel = 0;
  for (int i = 0; i < K; ++i) unrel += cs[i].rel < p.strong_rel;
  if (unrel == 0) return 0;
  auto w = std::make_shared<SbWait>();
  w->node = node;
  w->at = me;
  w->bound = bound;
  for (int i = 0; i < K; ++i) {
    w->cand.push_back(cs[i].v);
    w->zc.push_back(z[cs[i].v]);
    w->est[0].push_back(cs[i].e0);
    w->est[1].push_back(cs[i].e1);
    w->probed.push_back(cs[i].rel < p.strong_rel);
  }
  for (int d = 0; d < 2; ++d) {
    w->res[d].assign(K, std::numeric_limits<double>::quiet_NaN());
    w->src[d].assign(K, Parent{});
  }
  for (int i = 0; i < K; ++i) {
    if (!w->probed[i]) continue;
    for (int d = 1; d >= 0; --d) {
      auto pr = std::make_shared<Node>();
      pr->idx = node->idx;
      pr->idx.push_back(w->cand[i]);
      pr->val = node->val;
      pr->val.push_back((double)d);
      pr->bound = bound;
      pr->kind = STRONG;
      pr->parent = me;
      pr->depth = node->depth + 1;
      pr->bvar = w->cand[i];
      pr->bdir = d;
      pr->bfrac = std::max(1e-6, d ? 1.0 - w->zc[i] : w->zc[i]);
      pr->pbound = bound;
      pr->sb = w;
      pr->sb_i = i;
      strong_q.push_back(pr);
      w->pending += 1;
    }
  }
  sb_waiting += 1;
  st.strong_nodes += 1;
  return 1;
}

// all probes of a node are back: branch on the candidate with the best product of bound gains (a probe's bound is
// a valid bound of its child — the child inherits it; an infeasible / cut-off probe removes that child); both
// children of a candidate infeasible: the node's subtree is empty
void NepBnb::decide_strong(SbWait &w) {
  sb_waiting -= 1;
  const Node &node = *w.node;
  if (pruned(w.bound)) return;
  const double big = 1e30, eps = 1e-12;
  int best = -1;
  double bs = -1.0;
  for (size_t i = 0; i < w.cand.size(); ++i) {
    double g[2];
    for (int d = 0; d < 2; ++d) {
      if (w.probed[i]) {
        const double r = w.res[d][i];
        g[d] = (!(r < INF) || pruned(r)) ? big : std::max(eps, r - w.bound);
      } else {
        g[d] = std::max(eps, w.est[d][i]);
      }
    }
    if (g[0] >= big && g[1] >= big) return;   // neither child exists: nothing below this node
    const double sc = g[0] * g[1];
    if (sc > bs) { bs = sc; best = (int)i; }
  }
  if (best < 0) return;
  const int var = w.cand[best];
  st.strong_decided += 1;
  for (double v : {1.0, 0.0}) {
    const int d = v > 0.5 ? 1 : 0;
    double cb = w.bound;
    Parent src = w.at;
    if (w.probed[best]) {
      const double r = w.res[d][best];
      if (!(r < INF)) continue;                 // the probe proved this child infeasible / above the cutoff
      cb = std::max(cb, r);
      if (w.src[d][best].eng) src = w.src[d][best];
    }
    auto ch = std::make_shared<Node>();
    ch->idx = node.idx;
    ch->idx.push_back(var);
    ch->val = node.val;
    ch->val.push_back(v);
    ch->bound = std::max(cb, ibound(ch->idx, ch->val));
    ch->bvar = var;
    ch->bdir = d;
    ch->bfrac = std::max(1e-6, d ? 1.0 - w.zc[best] : w.zc[best]);
    ch->pbound = w.bound;
    if (pruned(ch->bound)) continue;
    ch->kind = (int)ch->idx.size() >= nb() ? LEAF : NODE;
    ch->parent = src;
    ch->depth = node.depth + 1;
    push_heap(ch);
  }
}

int NepBnb::branch_var_pc(const Node &node, const float *flow, const double *z) const {
  const int FN = p.F * p.N;
  std::vector<char> fixed(std::max(p.c1, p.n1) + 1, 0);
  for (int32_t i : node.idx) fixed[i] = 1;
  double avg[2][2];
  for (int k = 0; k < 2; ++k)
    for (int d = 0; d < 2; ++d)
      avg[k][d] = pck_cnt[k][d] > 0 ? pck_sum[k][d] / (double)pck_cnt[k][d]
                                    : (pck_cnt[k][1 - d] > 0 ? pck_sum[k][1 - d] / (double)pck_cnt[k][1 - d] : 1.0);
  const bool have = !pc_sum[0].empty();
  auto psi = [&](int v, int d, int k) {
    return (have && pc_cnt[d][v] > 0) ? pc_sum[d][v] / (double)pc_cnt[d][v] : avg[k][d];
  };
  const double eps = 1e-6, ftol = 1e-4;
  int best = -1;
  double bs = -1.0;
  auto consider = [&](int v, int k) {
    const double zf = z[v];
    if (!(zf > ftol && zf < 1.0 - ftol)) return;
    const double sc = std::max(psi(v, 0, k) * zf, eps) * std::max(psi(v, 1, k) * (1.0 - zf), eps);
    if (sc > bs) { bs = sc; best = v; }
  };
  if (p.n0 >= 0)
    for (int v = p.n0; v < p.n1; ++v)
      if (!fixed[v]) consider(v, 1);
  for (int q = 0; q < FN; ++q) {
    const int v = p.c0 + q;
    if (!fixed[v] && (double)flow[q] > p.flow_tol) consider(v, 0);
  }
  return best >= 0 ? best : branch_var(node, flow, z);
}

int NepBnb::branch_var(const Node &node, const float *flow, const double *z) const {
  const int F = p.F, N = p.N;
  std::vector<char> fixed(std::max(p.c1, p.n1) + 1, 0);
  for (int32_t i : node.idx) fixed[i] = 1;
  if (p.n0 >= 0) {
    int best = -1;
    double bv = -INF;
    for (int j = 0; j < N; ++j) {
      double in = 0.0;
      for (int f = 0; f < F; ++f) in += (double)flow[(size_t)f * N + j];
      if (!fixed[p.n0 + j] && in > p.flow_tol && in > bv) { bv = in; best = j; }
    }
    if (best >= 0) return p.n0 + best;
  }
  {
    int best = -1;
    double bv = -INF;
    for (int k = 0; k < F * N; ++k) {
      const double fl = (double)flow[k];
      if (!fixed[p.c0 + k] && fl > p.flow_tol && fl > bv) { bv = fl; best = k; }
    }
    if (best >= 0) return p.c0 + best;
  }
  int best = -1;
  double bv = -INF;
  for (int k = p.c0; k < p.c1; ++k)
    if (!fixed[k] && z[k] > bv) { bv = z[k]; best = k; }
  if (p.n0 >= 0)
    for (int k = p.n0; k < p.n1; ++k)
      if (!fixed[k] && z[k] > bv) { bv = z[k]; best = k; }
  return best;
}

// NeptuneStep2Base.integer_bound (core/solvers/neptune/neptune_step.py): the step-2 objective over integral
// placements bounded from a node's c (and n) fixings — additions A, removals R, the K-node cap; +inf when the
// fixings admit no integral completion; -inf without step 2
static double step2_ibound(const nep_bnb_params &p, bool s2_create, double s2_cap, const std::vector<char> &s2_old,
                           const std::vector<int32_t> &idx, const std::vector<double> &val);

double NepBnb::ibound(const std::vector<int32_t> &idx, const std::vector<double> &val) const {
  if (!s2) return -INF;
  return step2_ibound(p, s2_create, s2_cap, s2_old, idx, val);
}

static double step2_ibound(const nep_bnb_params &p, bool s2_create, double s2_cap, const std::vector<char> &s2_old,
                           const std::vector<int32_t> &idx, const std::vector<double> &val) {
  const int F = p.F, N = p.N, FN = F * N;
  const double w = (double)FN;
  std::vector<double> fx(FN, -1.0), nf(N, -1.0);
  for (size_t q = 0; q < idx.size(); ++q) {
    if (idx[q] >= p.c0 && idx[q] < p.c0 + FN) fx[idx[q] - p.c0] = val[q];
    else if (p.n0 >= 0 && idx[q] >= p.n0 && idx[q] < p.n1) nf[idx[q] - p.n0] = val[q];
  }
  std::vector<char> one(FN), zero(FN);
  double O = 0.0, add_fixed = 0.0, rem_fixed = 0.0;
  for (int k = 0; k < FN; ++k) {
    one[k] = fx[k] > 0.5;
    zero[k] = fx[k] >= 0 && fx[k] < 0.5;
    O += s2_old[k] ? 1.0 : 0.0;
    if (one[k] && !s2_old[k]) add_fixed += 1.0;
    if (zero[k] && s2_old[k]) rem_fixed += 1.0;
  }
  double uncovered = 0.0;
  std::vector<char> freef(F, 1);
  std::vector<double> ones_f(F, 0.0);
  for (int f = 0; f < F; ++f) {
    bool cov = false;
    for (int j = 0; j < N; ++j) {
      const int k = f * N + j;
      cov |= one[k] || (s2_old[k] && !zero[k]);
      if (one[k]) { freef[f] = 0; ones_f[f] += 1.0; }
    }
    if (!cov) uncovered += 1.0;
  }
  double A = add_fixed + uncovered, R_lb = rem_fixed;
  if (std::isfinite(s2_cap)) {
    const int K = (int)std::floor(s2_cap + 1e-9);
    std::vector<char> opened(N, 0), closed(N, 0);
    int n_open = 0;
    for (int j = 0; j < N; ++j) {
      bool any = false;
      for (int f = 0; f < F; ++f) any |= one[f * N + j] != 0;
      opened[j] = nf[j] > 0.5 || any;
      closed[j] = nf[j] >= 0 && nf[j] < 0.5;
      if (opened[j] && closed[j]) return INF;
      n_open += opened[j];
    }
    if (n_open > K) return INF;
    auto top_sum = [&](const std::vector<double> &v) {   // sum over opened + the K - n_open largest free others
      double s = 0.0;
      std::vector<double> rest;
      for (int j = 0; j < N; ++j) {
        if (opened[j]) s += v[j];
        else if (!closed[j]) rest.push_back(v[j]);
      }
      std::sort(rest.begin(), rest.end(), std::greater<double>());
      const int take = std::max(0, K - n_open);
      for (int q = 0; q < take && q < (int)rest.size(); ++q) s += rest[q];
      return s;
    };
    std::vector<double> keep(N, 0.0), cov(N, 0.0);
    double nfreef = 0.0;
    for (int f = 0; f < F; ++f) nfreef += freef[f];
    for (int j = 0; j < N; ++j) {
      if (closed[j]) continue;
      for (int f = 0; f < F; ++f) {
        const int k = f * N + j;
        if (s2_old[k] && !zero[k]) {
          keep[j] += 1.0;
          if (freef[f]) cov[j] += 1.0;
        }
      }
    }
    R_lb = std::max(R_lb, O - top_sum(keep));
    A = std::max(A, add_fixed + std::max(0.0, nfreef - top_sum(cov)));
  }
  if (s2_create) {
    double nzero = 0.0;
    for (int k = 0; k < FN; ++k) nzero += zero[k];
    if ((double)FN - nzero < O) return INF;
    return A + (2 * w - 1) * R_lb;
  }
  double need = 0.0, nfree = 0.0, kept = 0.0;
  for (int f = 0; f < F; ++f) {
    need += std::max(ones_f[f], 1.0);
    if (ones_f[f] == 0.0) nfree += 1.0;
  }
  if (need > O + 1e-9) return INF;
  for (int k = 0; k < FN; ++k) kept += (one[k] && s2_old[k]) ? 1.0 : 0.0;
  kept += std::max(0.0, nfree - (A - add_fixed));
  return (2 * w + 1) * A - (O - kept);
}

void NepBnb::round_all(const Node &node, const float *flow, const double *z, double bound, const Parent &me) {
  const int F = p.F, N = p.N, FN = F * N;
  std::vector<double> cfix(FN, -1.0), nfix;
  if (p.n0 >= 0) nfix.assign(N, -1.0);
  for (size_t q = 0; q < node.idx.size(); ++q) {
    const int i = node.idx[q];
    if (i >= p.c0 && i < p.c1) cfix[i - p.c0] = node.val[q];
    else if (p.n0 >= 0 && i >= p.n0 && i < p.n1) nfix[i - p.n0] = node.val[q];
  }
  const int modes = p.unit_flow_leaves ? 3 : 2;
  const int32_t by_flow[3] = {0, 1, 1};
  const double thr[3] = {p.flow_tol, p.flow_tol, 1.0 - 1e-6};
  std::vector<double> cout((size_t)modes * FN), nout(p.n0 >= 0 ? (size_t)modes * N : 0);
  int32_t found[3] = {0, 0, 0};
  if (nep_round_leaves(F, N, cfix.data(), p.n0 >= 0 ? nfix.data() : nullptr, flow, z + p.c0, fn_mem.data(),
                       node_mem.data(), modes, by_flow, thr, cout.data(), p.n0 >= 0 ? nout.data() : nullptr,
                       found) < 0)
    return;
  for (int q = 0; q < modes; ++q) {
    if (!found[q]) continue;
    auto leaf = std::make_shared<Node>();
    leaf->kind = LEAF;
    leaf->parent = me;
    leaf->depth = node.depth + 1;
    if (leaf_idx.empty()) {   // (every rounding leaf fixes the same variables: every c, then every n)
      for (int k = p.c0; k < p.c1; ++k) leaf_idx.push_back(k);
      if (p.n0 >= 0)
        for (int k = p.n0; k < p.n1; ++k) leaf_idx.push_back(k);
    }
    leaf->idx = leaf_idx;
    leaf->val.reserve(leaf_idx.size());
    leaf->val.assign(cout.begin() + (size_t)q * FN, cout.begin() + (size_t)(q + 1) * FN);
    if (p.n0 >= 0) leaf->val.insert(leaf->val.end(), nout.begin() + (size_t)q * N, nout.begin() + (size_t)(q + 1) * N);
    if (!seen.insert(key_of(leaf->val)).second) continue;
    leaf->bound = std::max(bound, ibound(leaf->idx, leaf->val));
    if (!pruned(leaf->bound)) pending.push_back(leaf);
  }
}

int NepBnb::finish_one(Engine &eng, int slot, const NodeP &node, int status, double o, double po, int64_t iters,
                       const float *flow, const double *z) {
  eng.inflight -= 1;
  st.lp_iterations += iters;
  lp_iters.push_back(iters);
  const int col = status_col(status);
  if (node->kind == STRONG) {   // a strong-branching probe: its bound (or infeasibility) for the waiting node
    st.strong_lps += 1;
    st.strong_iterations += iters;
    const bool gone = status == NEP_LP_INFEASIBLE || status == NEP_LP_CUTOFF;
    pc_update(*node, gone ? incv() : o);
    SbWait &w = *node->sb;
    const int d = node->bdir, i = node->sb_i;
    w.res[d][i] = gone ? INF : std::max(node->pbound, o);
    if (!gone) w.src[d][i] = Parent{&eng, slot, eng.gen[slot]};
    eng.free.push_back(slot);
    if (--w.pending == 0) decide_strong(w);
    return NEP_OK;
  }
  st.lp_status[col] += 1;
  st.lp_status_kind[node->kind][col] += 1;
  if (node->kind == REFROOT) {
    if (p.warm && status != NEP_LP_INFEASIBLE && status != NEP_LP_CUTOFF) {
      int rc = eng.ops.copy_state(eng.ops.ctx, slot, eng.root_slot);
      if (rc) return rc;
      eng.root_state = true;
    }
    eng.root_ready = true;
    eng.free.push_back(slot);
    return NEP_OK;
  }
  if (status == NEP_LP_OPTIMAL) st.certified += 1;
  if (p.branching >= 1 && node->kind == NODE)   // (an infeasible / cut-off child gained up to the incumbent)
    pc_update(*node, (status == NEP_LP_INFEASIBLE || status == NEP_LP_CUTOFF) ? incv() : o);
  if (!eng.root_ready && node->depth == 0 && node->kind == NODE) {
    st.root_seconds = now_s() - t0;
    if (p.warm && status != NEP_LP_INFEASIBLE && status != NEP_LP_CUTOFF) {
      int rc = eng.ops.copy_state(eng.ops.ctx, slot, eng.root_slot);
      if (rc) return rc;
      eng.root_state = true;
    }
    eng.root_ready = true;
    const Parent me0{&eng, slot, eng.gen[slot]};
    for (auto &s : seeds) {
      s->bound = ibound(s->idx, s->val);
      if (!(s->bound < INF)) continue;
      if (!seen.insert(key_of(s->val)).second) continue;
      s->parent = me0;
      s->depth = 1;
      pending.push_back(s);
    }
    seeds.clear();
  }
  if (status == NEP_LP_INFEASIBLE || status == NEP_LP_CUTOFF) {
    eng.free.push_back(slot);
    return NEP_OK;
  }
  const double bound = std::max(node->bound, o);
  if (node->kind != NODE) {
    st.leaves += 1;
    bool kept = false;
    if (status == NEP_LP_OPTIMAL) {
      if (po < incv() - gap_abs(incv())) {
        inc = po;
        inc_source = 1;
        inc_node = node;
        inc_z.assign(eng.n_int, 0.0);
        int rc = eng.ops.get_solutions(eng.ops.ctx, 1, &slot, inc_z.data());
        if (rc) return rc;
        if (p.warm) {
          rc = eng.ops.copy_state(eng.ops.ctx, slot, eng.inc_slot);
          if (rc) return rc;
          inc_slot = eng.inc_slot;
        } else {
          if (keep_slot >= 0) eng.free.push_back(keep_slot);
          keep_slot = slot;
          inc_slot = slot;
          kept = true;
        }
        st.lp_incumbents += 1;
        rc = set_cutoffs();
        if (rc) return rc;
        if (inc_events) inc_queue.push_back(IncEvent{node, Parent{&eng, slot, eng.gen[slot]}, po});
      }
    } else if (node->kind == LEAF) {
      double pres = 0.0;
      if (std::isfinite(p.retry_res)) {
        double d[16];
        int rc = eng.ops.get_diag(eng.ops.ctx, slot, d);
        if (rc) return rc;
        pres = d[3];
      }
      if (pres <= p.retry_res) {
        auto r = std::make_shared<Node>(*node);
        r->bound = bound;
        r->kind = RETRY;
        r->parent = Parent{&eng, slot, eng.gen[slot]};
        retry.push_back(r);
      } else {
        st.unresolved += 1;
        unresolved_bounds.push_back(bound);
      }
    } else {
      st.unresolved += 1;
      unresolved_bounds.push_back(bound);
    }
    if (!kept) eng.free.push_back(slot);
    return NEP_OK;
  }
  if (pruned(bound)) {
    eng.free.push_back(slot);
    return NEP_OK;
  }
  st.nodes += 1;
  const Parent me{&eng, slot, eng.gen[slot]};
  {
    const double t0 = prof ? now_s() : 0.0;
    round_all(*node, flow, z, bound, me);
    if (prof) { pr_round += now_s() - t0; ++pr_rounds; }
  }
  if (p.primal_at_root && node->depth == 0 && !root_event_done) {
    // the caller's primal heuristic runs on this node's LP (z, flows) before the search goes on
    root_event_pending = true;
    ev_z.assign(z, z + eng.n_int);
    ev_flow.assign(flow, flow + (size_t)p.F * p.N);
    ev_node = node;
    ev_parent = me;
    ev_bound = bound;
  }
  if (p.branching == 2 && start_strong(node, flow, z, bound, me)) {
    eng.free.push_back(slot);   // (its probes warm-start from this slot; they are submitted first)
    return NEP_OK;
  }
  const int var = p.branching >= 1 ? branch_var_pc(*node, flow, z) : branch_var(*node, flow, z);
  if (var >= 0) {
    for (double v : {1.0, 0.0}) {
      auto ch = std::make_shared<Node>();
      ch->idx = node->idx;
      ch->idx.push_back(var);
      ch->val = node->val;
      ch->val.push_back(v);
      ch->bound = std::max(bound, ibound(ch->idx, ch->val));
      ch->bvar = var;
      ch->bdir = v > 0.5 ? 1 : 0;
      ch->bfrac = std::max(1e-6, v > 0.5 ? 1.0 - z[var] : z[var]);
      ch->pbound = bound;
      if (pruned(ch->bound)) continue;
      ch->kind = (int)ch->idx.size() >= nb() ? LEAF : NODE;
      ch->parent = me;
      ch->depth = node->depth + 1;
      push_heap(ch);
    }
  }
  eng.free.push_back(slot);   // most recently finished last: its state survives longest
  return NEP_OK;
}

// every finished LP of one advance of `eng`: the flows / integer vectors of the branching nodes that will
// branch, read in one device call each, then each LP in order
int NepBnb::finish_block(Engine &eng, int nd) {
  std::vector<int32_t> want;
  for (int i = 0; i < nd; ++i) {
    const NodeP &node = eng.running[done_slots[i]];
    if (!node || node->kind != NODE || sts[i] == NEP_LP_INFEASIBLE || sts[i] == NEP_LP_CUTOFF) continue;
    if (pruned(std::max(node->bound, obj[i]))) continue;
    want.push_back(done_slots[i]);
  }
  const size_t FN = (size_t)p.F * p.N;
  const int ni = eng.n_int;
  std::vector<float> fl(want.size() * FN);
  std::vector<double> zs(want.size() * ni);
  if (!want.empty()) {
    const double t0 = prof ? now_s() : 0.0;
    int rc;
    if (eng.ops.get_flows_solutions) {
      rc = eng.ops.get_flows_solutions(eng.ops.ctx, (int)want.size(), want.data(), fl.data(), zs.data());
    } else {
      rc = eng.ops.get_flows(eng.ops.ctx, (int)want.size(), want.data(), fl.data());
      if (!rc) rc = eng.ops.get_solutions(eng.ops.ctx, (int)want.size(), want.data(), zs.data());
    }
    if (rc) return rc;
    if (prof) { pr_reads += now_s() - t0; ++pr_reads_calls; }
  }
  // (copies: finish_one may submit nothing, but the outputs are reused by later advances)
  const std::vector<int32_t> ds(done_slots.begin(), done_slots.begin() + nd);
  const std::vector<int32_t> ss(sts.begin(), sts.begin() + nd);
  const std::vector<double> ob(obj.begin(), obj.begin() + nd), po(pobj.begin(), pobj.begin() + nd);
  const std::vector<int64_t> it(its.begin(), its.begin() + nd);
  for (int i = 0; i < nd; ++i) {
    const int slot = ds[i];
    NodeP node = eng.running[slot];
    eng.running[slot] = nullptr;
    if (!node) continue;
    const float *f = nullptr;
    const double *z = nullptr;
    for (size_t w = 0; w < want.size(); ++w)
      if (want[w] == slot) { f = fl.data() + w * FN; z = zs.data() + w * ni; }
    std::vector<float> fl1;
    std::vector<double> z1;
    if (node->kind == NODE && !f && ss[i] != NEP_LP_INFEASIBLE && ss[i] != NEP_LP_CUTOFF &&
        !pruned(std::max(node->bound, ob[i]))) {
      // (the incumbent improved within this block: read it now)
      fl1.resize(FN);
      z1.resize(ni);
      int rc = eng.ops.get_flows_solutions ? eng.ops.get_flows_solutions(eng.ops.ctx, 1, &slot, fl1.data(), z1.data())
                                           : eng.ops.get_flows(eng.ops.ctx, 1, &slot, fl1.data());
      if (!rc && !eng.ops.get_flows_solutions) rc = eng.ops.get_solutions(eng.ops.ctx, 1, &slot, z1.data());
      if (rc) return rc;
      f = fl1.data();
      z = z1.data();
    }
    const double t0 = prof ? now_s() : 0.0;
    int rc = finish_one(eng, slot, node, ss[i], ob[i], po[i], it[i], f, z);
    if (prof) pr_finish += now_s() - t0;
    if (rc) return rc;
  }
  return NEP_OK;
}

int NepBnb::drain_and_close() {
  const double t = now_s();
  std::vector<double> open;
  for (int e = 0; e < n_engines(); ++e)
    for (auto &n : engines[e]->running)
      if (n && n->kind != REFROOT) open.push_back(n->bound);
  st.drained = (int64_t)open.size();
  for (int e = 0; e < n_engines(); ++e) {
    const nep_bnb_engine &o = engines[e]->ops;
    if (o.active(o.ctx) > 0) {
      const int rc = o.set_params(o.ctx, p.tol, -INF);
      if (rc) return rc;
    }
  }
  for (int e = 0; e < n_engines(); ++e) {
    Engine &eng = *engines[e];
    const nep_bnb_engine &o = eng.ops;
    while (o.active(o.ctx) > 0) {
      int32_t nd = 0;
      int rc = o.advance(o.ctx, o.active(o.ctx), &nd, done_slots.data(), obj.data(), pobj.data(), sts.data(),
                         its.data());
      if (rc) return rc;
      for (int i = 0; i < nd; ++i) {
        NodeP n = eng.running[done_slots[i]];
        eng.running[done_slots[i]] = nullptr;
        if (n && n->kind != REFROOT && sts[i] != NEP_LP_INFEASIBLE) open.push_back(std::max(n->bound, obj[i]));
      }
    }
  }
  st.drain_seconds = now_s() - t;
  while (!heap.empty()) { open.push_back(heap.top().bound); heap.pop(); }
  for (auto &n : pending) open.push_back(n->bound);
  for (auto &n : retry) open.push_back(n->bound);
  for (auto &n : strong_q) open.push_back(n->bound);
  for (double b : unresolved_bounds) open.push_back(b);
  double bound = incv();
  for (double b : open) bound = std::min(bound, b);
  st.bound = bound;
  st.any_unresolved = unresolved_bounds.empty() ? 0 : 1;
  st.unresolved_below = 0;
  for (double b : unresolved_bounds)
    if (b < incv() - gap_abs(incv())) st.unresolved_below = 1;
  st.limit_hit = limit_hit ? 1 : 0;
  st.stalled = stalled ? 1 : 0;
  st.incumbent = inc;
  st.agreed_incumbent = incv();
  st.incumbent_source = inc_source;
  st.incumbent_slot = inc_source == 1 ? inc_slot : -1;
  finished = true;
  return NEP_OK;
}

// the sharded search's split (bnb.py solve): the frontier — identical on every rank — in canonical order
// (bound, -depth, seq), its crc32, then every rank keeps the open nodes whose position is its rank mod world
void NepBnb::deal_frontier() {
  std::vector<HeapItem> items;
  while (!heap.empty()) {
    items.push_back(heap.top());
    heap.pop();
  }
  std::sort(items.begin(), items.end(), [](const HeapItem &a, const HeapItem &b) { return b > a; });
  uint32_t h = 0;
  for (const auto &it : items) {
    const double bd[2] = {it.bound, (double)it.negdepth};
    h = crc32_update(h, bd, sizeof bd);
    std::vector<int64_t> ix(it.node->idx.begin(), it.node->idx.end());
    h = crc32_update(h, ix.data(), ix.size() * sizeof(int64_t));
    h = crc32_update(h, it.node->val.data(), it.node->val.size() * sizeof(double));
  }
  st.split_hash = h;
  for (size_t i = 0; i < items.size(); ++i)
    if ((int)(i % (size_t)p.world) == p.rank) heap.push(items[i]);
  auto keep = [&](std::deque<NodeP> &q) {
    std::deque<NodeP> out;
    for (size_t i = 0; i < q.size(); ++i)
      if ((int)(i % (size_t)p.world) == p.rank) out.push_back(q[i]);
    q.swap(out);
  };
  keep(pending);
  keep(retry);
  st.presplit_nodes = st.nodes;
  st.presplit_lps = st.lps;
  st.presplit_certified = st.certified;
  split = true;
}

// the k best-bound open nodes, taken off this rank's heap for another rank (bnb.py _rebalance's donor side)
int NepBnb::export_nodes(int k, int32_t cap, int32_t *lens, double *meta, int32_t *idx, double *val) {
  int32_t used = 0;
  for (int q = 0; q < k; ++q) {
    if (heap.empty()) return bad(NEP_ERR_ARG, "nep_bnb_export_nodes: fewer open nodes than asked for");
    const NodeP n = heap.top().node;
    const int32_t len = (int32_t)n->idx.size();
    if (used + len > cap) return bad(NEP_ERR_ARG, "nep_bnb_export_nodes: idx / val capacity too small");
    heap.pop();
    lens[q] = len;
    meta[3 * q] = n->bound;
    meta[3 * q + 1] = n->depth;
    meta[3 * q + 2] = n->kind;
    std::copy(n->idx.begin(), n->idx.end(), idx + used);
    std::copy(n->val.begin(), n->val.end(), val + used);
    used += len;
  }
  return NEP_OK;
}

extern "C" {

void *nep_bnb_create_engines(const nep_bnb_engine *leaf, const nep_bnb_engine *bound, const nep_bnb_params *params,
                             const double *fn_mem, const double *node_mem) {
  if (!leaf || !params || !fn_mem || !node_mem) {
    bad(NEP_ERR_ARG, "nep_bnb_create: null argument");
    return nullptr;
  }
  if (!ops_complete(*leaf) || (bound && !ops_complete(*bound))) {
    bad(NEP_ERR_ARG, "nep_bnb_create: incomplete engine call table");
    return nullptr;
  }
  const nep_bnb_params &q = *params;
  if (q.batch < 1 || (bound && q.batch_b < 1) || q.F < 1 || q.N < 1 || q.c0 < 0 || q.c1 > leaf->n_int ||
      (q.n0 >= 0 && q.n1 > leaf->n_int)) {
    bad(NEP_ERR_ARG, "nep_bnb_create: bad batch / layout parameters");
    return nullptr;
  }
  if (q.world < 1 || q.rank < 0 || q.rank >= q.world) {
    bad(NEP_ERR_ARG, "nep_bnb_create: bad world / rank");
    return nullptr;
  }
  auto *t = new NepBnb();
  {
    const char *e = std::getenv("NEP_BNB_PROFILE");
    t->prof = e && e[0] == '1';
  }
  t->p = *params;
  t->two = bound != nullptr;
  t->fn_mem.assign(fn_mem, fn_mem + params->F);
  t->node_mem.assign(node_mem, node_mem + params->N);
  init_engine(t->L, *leaf, 2);   // (bnb.py: root and incumbent slots whenever max_batch >= 3)
  t->engines[0] = &t->L;
  if (t->two) {
    init_engine(t->B, *bound, t->p.warm ? 1 : 0);
    t->engines[0] = &t->B;   // (bnb.py's engine order: bound model first)
    t->engines[1] = &t->L;
  }
  if (t->L.free.empty() || (t->two && t->B.free.empty())) {
    delete t;
    bad(NEP_ERR_ARG, "nep_bnb_create: no working slot left after the reserved ones (max_batch too small)");
    return nullptr;
  }
  const int mb = std::max(t->L.max_batch, t->two ? t->B.max_batch : 0);
  t->done_slots.assign(mb, 0);
  t->sts.assign(mb, 0);
  t->obj.assign(mb, 0.0);
  t->pobj.assign(mb, 0.0);
  t->its.assign(mb, 0);
  // the root (the heap) and, with two models and warm starts, the reference root the leaves start from
  auto root = std::make_shared<Node>();
  root->bound = -INF;
  root->kind = NODE;
  root->depth = 0;
  t->push_heap(root);
  if (t->two) {
    if (t->p.warm) {
      t->refroot = std::make_shared<Node>();
      t->refroot->bound = -INF;
      t->refroot->kind = REFROOT;
      t->refroot->depth = 0;
    } else {
      t->L.root_ready = true;
    }
  }
  return t;
}

void *nep_bnb_create(void *leaf_model, void *bound_model, const nep_bnb_params *params, const double *fn_mem,
                     const double *node_mem) {
  if (!leaf_model) {
    bad(NEP_ERR_ARG, "nep_bnb_create: null leaf model");
    return nullptr;
  }
  nep_bnb_engine le{}, be{};
  if (model_ops(leaf_model, &le)) return nullptr;   // (nep_model_get_info set the message)
  if (bound_model && model_ops(bound_model, &be)) return nullptr;
  return nep_bnb_create_engines(&le, bound_model ? &be : nullptr, params, fn_mem, node_mem);
}

void nep_bnb_destroy(void *tree) { delete static_cast<NepBnb *>(tree); }

int nep_bnb_add_leaf(void *tree, int32_t n, const int32_t *idx, const double *val, double bound, int32_t where) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || n < 0 || (n > 0 && (!idx || !val))) return bad(NEP_ERR_ARG, "nep_bnb_add_leaf: bad argument");
  for (int32_t q = 0; q < n; ++q)
    if (idx[q] < 0 || idx[q] >= t->L.n_int) return bad(NEP_ERR_ARG, "nep_bnb_add_leaf: index out of range");
  auto leaf = std::make_shared<Node>();
  leaf->idx.assign(idx, idx + n);
  leaf->val.assign(val, val + n);
  leaf->kind = LEAF;
  leaf->bound = bound;
  if (where == 0) {   // a seed leaf: queued when the root LP finishes
    leaf->depth = 1;
    t->seeds.push_back(leaf);
    return NEP_OK;
  }
  if (where == 2) {   // a neighbour of the NEP_BNB_INCUMBENT event's leaf: its own bound, at the front
    if (!t->seen.insert(NepBnb::key_of(leaf->val)).second) return NEP_OK;
    leaf->bound = std::max(bound, t->ibound(leaf->idx, leaf->val));
    leaf->parent = t->cur_inc.at;
    leaf->depth = t->cur_inc.node ? t->cur_inc.node->depth : 1;
    t->pending.push_front(leaf);
    return NEP_OK;
  }
  // where = 1: a leaf of the root event's node (the primal heuristic), at the front of the leaf queue
  if (!t->seen.insert(NepBnb::key_of(leaf->val)).second) return NEP_OK;
  leaf->bound = std::max(std::max(t->ev_bound, bound), t->ibound(leaf->idx, leaf->val));
  leaf->parent = t->ev_parent;
  leaf->depth = t->ev_node ? t->ev_node->depth + 1 : 1;
  if (!t->pruned(leaf->bound)) t->pending.push_front(leaf);
  return NEP_OK;
}

int nep_bnb_set_step2(void *tree, int32_t create, double node_cap, const double *old_alloc, int32_t incumbent_events) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !old_alloc || t->started) return bad(NEP_ERR_ARG, "nep_bnb_set_step2: bad argument or search started");
  const size_t FN = (size_t)t->p.F * t->p.N;
  t->s2 = true;
  t->s2_create = create != 0;
  t->s2_cap = node_cap;
  t->s2_old.resize(FN);
  for (size_t k = 0; k < FN; ++k) t->s2_old[k] = old_alloc[k] > 0.5;
  t->inc_events = incumbent_events != 0;
  // the root's bound is the integer bound of the empty box (+inf: no integral point at all)
  const double rb = t->ibound({}, {});
  while (!t->heap.empty()) t->heap.pop();
  if (rb < INF) {
    auto root = std::make_shared<Node>();
    root->bound = rb;
    root->kind = NODE;
    root->depth = 0;
    t->push_heap(root);
  }
  return NEP_OK;
}

int nep_bnb_debug_ibound(const nep_bnb_params *params, int32_t create, double node_cap, const double *old_alloc,
                         int32_t n, const int32_t *idx, const double *val, double *out) {
  if (!params || !old_alloc || !out || n < 0 || (n > 0 && (!idx || !val)))
    return bad(NEP_ERR_ARG, "nep_bnb_debug_ibound: bad argument");
  const size_t FN = (size_t)params->F * params->N;
  std::vector<char> old(FN);
  for (size_t k = 0; k < FN; ++k) old[k] = old_alloc[k] > 0.5;
  *out = step2_ibound(*params, create != 0, node_cap, old, std::vector<int32_t>(idx, idx + n),
                      std::vector<double>(val, val + n));
  return NEP_OK;
}

int nep_bnb_incumbent_event(void *tree, int32_t *n_fix, int32_t *idx, double *val, double *value) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !t->cur_inc.node) return bad(NEP_ERR_STATE, "nep_bnb_incumbent_event: no incumbent event");
  const Node &nd = *t->cur_inc.node;
  if (n_fix) *n_fix = (int32_t)nd.idx.size();
  if (idx) std::memcpy(idx, nd.idx.data(), nd.idx.size() * sizeof(int32_t));
  if (val) std::memcpy(val, nd.val.data(), nd.val.size() * sizeof(double));
  if (value) *value = t->cur_inc.value;
  return NEP_OK;
}

int nep_bnb_set_incumbent(void *tree, double value) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t) return bad(NEP_ERR_ARG, "nep_bnb_set_incumbent: null tree");
  if (!(value < t->inc)) return NEP_OK;
  t->inc = value;
  t->inc_source = 2;
  if (t->keep_slot >= 0) {
    t->L.free.push_back(t->keep_slot);
    t->keep_slot = -1;
  }
  t->inc_slot = -1;
  t->inc_node = nullptr;
  t->st.heuristic_incumbents += 1;
  return t->set_cutoffs();
}

int nep_bnb_event_data(void *tree, double *z, float *flow) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || t->ev_z.empty()) return bad(NEP_ERR_STATE, "nep_bnb_event_data: no root event");
  if (z) std::memcpy(z, t->ev_z.data(), t->ev_z.size() * sizeof(double));
  if (flow) std::memcpy(flow, t->ev_flow.data(), t->ev_flow.size() * sizeof(float));
  return NEP_OK;
}

int nep_bnb_run(void *tree, int32_t *event) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !event) return bad(NEP_ERR_ARG, "nep_bnb_run: null argument");
  *event = NEP_BNB_DONE;
  if (t->finished) return NEP_OK;
  if (!t->started) {
    t->started = true;
    t->t0 = now_s();
  }
  NepBnb &T = *t;
  Engine &L = T.L, &B = T.B;
  for (;;) {
    if (!T.inc_queue.empty()) {   // the caller's neighbours of a new LP incumbent (step 2's node relocation)
      T.cur_inc = T.inc_queue.front();
      T.inc_queue.pop_front();
      *event = NEP_BNB_INCUMBENT;
      return NEP_OK;
    }
    if (T.root_event_pending) {   // the caller's primal heuristic on the root node
      T.root_event_pending = false;
      T.root_event_done = true;
      *event = NEP_BNB_ROOT;
      return NEP_OK;
    }
    const bool sharded = T.p.world > 1;
    if (sharded && !T.split && T.heap.size() >= (size_t)T.p.world * (size_t)T.p.batch && L.inflight == 0 &&
        (!T.two || B.inflight == 0) && T.strong_q.empty() && T.sb_waiting == 0)
      T.deal_frontier();   // the frontier every rank holds identically, dealt once
    bool stop = T.stalled || T.st.nodes >= T.p.node_limit ||
                (T.p.time_limit > 0 && now_s() - T.t0 > T.p.time_limit);
    int busy = 0;
    for (int e = 0; e < T.n_engines(); ++e)
      for (auto &n : T.engines[e]->running)
        if (n && n->kind != REFROOT) ++busy;
    int64_t open_n = (int64_t)(T.heap.size() + T.pending.size() + T.retry.size() + T.strong_q.size()) + busy;
    if (sharded) {
      // one collective per loop, run by the caller: incumbent MIN, stop OR, open + in-flight SUM
      if (!T.sync_answered) {
        const double out[6] = {T.incv(), stop ? 1.0 : 0.0, (double)open_n, (double)T.heap.size(),
                               T.split ? 1.0 : 0.0, (double)T.st.sync_calls};
        std::copy(out, out + 6, T.sync_out);
        *event = NEP_BNB_SYNC;
        return NEP_OK;
      }
      T.sync_answered = false;
      stop = T.agreed_stop;
      if (T.split) open_n = T.agreed_open;   // (before the split every rank holds the same open nodes)
    }
    if (open_n == 0) break;
    if (stop) {
      T.limit_hit = true;
      break;
    }
    // fill the free slots: retries, rounding leaves, then best-first open nodes
    std::vector<std::pair<Engine *, std::pair<int, NodeP>>> items;
    // at most `batch` LPs in flight per model; further free slots keep finished states (parked parents)
    int capL = T.p.batch - L.inflight, capB = T.p.batch_b - B.inflight;
    if (!T.two) {
      while (!L.free.empty() && capL > 0 &&
             (!T.strong_q.empty() || !T.retry.empty() || !T.pending.empty() || !T.heap.empty())) {
        NodeP node;
        if (!T.strong_q.empty()) {   // strong-branching probes first: their node waits for them
          node = T.strong_q.front();
          T.strong_q.pop_front();
        } else if (!T.retry.empty()) {
          node = T.retry.front();
          T.retry.pop_front();
        } else if (!T.pending.empty()) {
          node = T.pending.front();
          T.pending.pop_front();
          if (T.pruned(node->bound)) continue;
        } else {
          node = T.heap.top().node;
          T.heap.pop();
          if (T.pruned(node->bound)) continue;
        }
        const int s = L.free.front();
        L.free.pop_front();
        items.push_back({&L, {s, node}});
        --capL;
        if (!L.root_ready) break;   // the root runs alone (its state warm-starts everything after)
      }
    } else {
      if (T.refroot && !L.free.empty() && capL > 0) {
        const int s = L.free.front();
        L.free.pop_front();
        --capL;
        items.push_back({&L, {s, T.refroot}});
        T.refroot = nullptr;
      }
      while (!B.free.empty() && capB > 0 && !T.strong_q.empty()) {   // probes of branching nodes first
        NodeP node = T.strong_q.front();
        T.strong_q.pop_front();
        const int s = B.free.front();
        B.free.pop_front();
        items.push_back({&B, {s, node}});
        --capB;
      }
      while (!B.free.empty() && capB > 0 && !T.heap.empty() && (!B.root_ready || L.root_ready)) {
        NodeP node = T.heap.top().node;
        T.heap.pop();
        if (T.pruned(node->bound)) continue;
        if (node->kind != NODE) {   // a leaf from branching: the reference model's
          T.pending.push_back(node);
          continue;
        }
        const int s = B.free.front();
        B.free.pop_front();
        items.push_back({&B, {s, node}});
        --capB;
        if (!B.root_ready) break;
      }
      while (L.root_ready && !L.free.empty() && capL > 0 && (!T.retry.empty() || !T.pending.empty())) {
        NodeP node;
        if (!T.retry.empty()) {
          node = T.retry.front();
          T.retry.pop_front();
        } else {
          node = T.pending.front();
          T.pending.pop_front();
        }
        if (node->kind == LEAF && T.pruned(node->bound)) continue;
        const int s = L.free.front();
        L.free.pop_front();
        --capL;
        items.push_back({&L, {s, node}});
      }
    }
    double t1 = now_s();
    if (!items.empty()) {
      int rc = T.submit(items);
      if (rc) return rc;
    }
    double t2 = now_s();
    T.st.submit_seconds += t2 - t1;
    int inflight = 0;
    for (int e = 0; e < T.n_engines(); ++e) inflight += T.engines[e]->inflight;
    if (inflight == 0) {
      // nothing iterates: either this rank's part of a sharded frontier is empty (the others still work), or
      // open nodes wait for a slot that never frees (round-5 ADVICE: e.g. warm starts off with one working slot
      // kept for the incumbent) — end the search as a limit instead of looping forever
      if (items.empty() && T.heap.size() + T.pending.size() + T.retry.size() + T.strong_q.size() > 0)
        T.stalled = true;
      continue;
    }
    T.st.advance_calls += 1;
    T.st.inflight_sum += busy;
    for (int e = 0; e < T.n_engines(); ++e) {
      Engine &eng = *T.engines[e];
      if (eng.inflight <= 0) continue;
      // before the split every rank must stay identical: drain each batch whole
      const int min_done = (sharded && !T.split) ? eng.inflight : (T.two ? 0 : (T.p.time_limit > 0 ? 0 : 1));
      int32_t nd = 0;
      int rc = eng.ops.advance(eng.ops.ctx, min_done, &nd, T.done_slots.data(), T.obj.data(), T.pobj.data(),
                               T.sts.data(), T.its.data());
      if (rc) return rc;
      const double t3 = now_s();
      T.st.advance_seconds += t3 - t2;
      rc = T.finish_block(eng, nd);
      if (rc) return rc;
      t2 = now_s();
      T.st.finish_seconds += t2 - t3;
    }
  }
  int rc = T.drain_and_close();
  if (rc) return rc;
  *event = NEP_BNB_DONE;
  return NEP_OK;
}

int nep_bnb_sync_get(void *tree, double *out6) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !out6) return bad(NEP_ERR_ARG, "nep_bnb_sync_get: null argument");
  std::copy(t->sync_out, t->sync_out + 6, out6);
  return NEP_OK;
}

int nep_bnb_sync_set(void *tree, double incumbent, int32_t stop, int64_t open_total) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t) return bad(NEP_ERR_ARG, "nep_bnb_sync_set: null tree");
  t->sync_answered = true;
  t->agreed_stop = stop != 0;
  t->agreed_open = open_total;
  t->st.sync_calls += 1;
  if (incumbent < t->cut) {
    const double before = t->incv();
    t->cut = incumbent;
    if (t->incv() < before) return t->set_cutoffs();
  }
  return NEP_OK;
}

int nep_bnb_export_nodes(void *tree, int32_t k, int32_t cap, int32_t *lens, double *meta, int32_t *idx, double *val) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || k < 0 || (k > 0 && (!lens || !meta || (cap > 0 && (!idx || !val)))))
    return bad(NEP_ERR_ARG, "nep_bnb_export_nodes: bad argument");
  return t->export_nodes(k, cap, lens, meta, idx, val);
}

int nep_bnb_import_nodes(void *tree, int32_t k, const int32_t *lens, const double *meta, const int32_t *idx,
                         const double *val) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || k < 0 || (k > 0 && (!lens || !meta))) return bad(NEP_ERR_ARG, "nep_bnb_import_nodes: bad argument");
  int64_t o = 0;
  for (int q = 0; q < k; ++q) {
    if (lens[q] < 0 || (lens[q] > 0 && (!idx || !val))) return bad(NEP_ERR_ARG, "nep_bnb_import_nodes: bad node");
    auto n = std::make_shared<Node>();
    n->idx.assign(idx + o, idx + o + lens[q]);
    n->val.assign(val + o, val + o + lens[q]);
    o += lens[q];
    for (int32_t i : n->idx)
      if (i < 0 || i >= t->L.n_int) return bad(NEP_ERR_ARG, "nep_bnb_import_nodes: index out of range");
    n->bound = meta[3 * q];
    n->depth = (int)meta[3 * q + 1];
    n->kind = (int)meta[3 * q + 2];
    // (no parent state on this rank: the node starts from its model's root state)
    if (!t->pruned(n->bound)) {
      t->push_heap(n);
      t->st.rebalanced += 1;
    }
  }
  return NEP_OK;
}

int nep_bnb_get_stats(void *tree, nep_bnb_stats *out) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !out) return bad(NEP_ERR_ARG, "nep_bnb_get_stats: null argument");
  *out = t->st;
  out->n_lp_iters = (int64_t)t->lp_iters.size();
  return NEP_OK;
}

int nep_bnb_get_lp_iters(void *tree, int64_t *out) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t || !out) return bad(NEP_ERR_ARG, "nep_bnb_get_lp_iters: null argument");
  if (!t->lp_iters.empty()) std::memcpy(out, t->lp_iters.data(), t->lp_iters.size() * sizeof(int64_t));
  return NEP_OK;
}

int nep_bnb_incumbent(void *tree, double *z, int32_t *n_fix, int32_t *idx, double *val) {
  auto *t = static_cast<NepBnb *>(tree);
  if (!t) return bad(NEP_ERR_ARG, "nep_bnb_incumbent: null tree");
  if (t->inc_source != 1 || !t->inc_node) {
    if (n_fix) *n_fix = -1;
    return NEP_OK;
  }
  if (z) std::memcpy(z, t->inc_z.data(), t->inc_z.size() * sizeof(double));
  if (n_fix) *n_fix = (int32_t)t->inc_node->idx.size();
  if (idx) std::memcpy(idx, t->inc_node->idx.data(), t->inc_node->idx.size() * sizeof(int32_t));
  if (val) std::memcpy(val, t->inc_node->val.data(), t->inc_node->val.size() * sizeof(double));
  return NEP_OK;
}

}  // extern "C"
