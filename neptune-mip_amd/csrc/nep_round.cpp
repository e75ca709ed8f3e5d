// nep_round.cpp — native rounding heuristic of the branch-and-bound (host code; include/neptune_lp.h
// nep_round_leaf).  One branching node's LP (its flows F x N and its c) -> a leaf fixing every c and n,
// the memory-aware greedy of core/engine/bnb.py (DESIGN.md §7 "Primal heuristic"), run per finished node
// (three modes each): in Python it was ~0.1 ms a call and ~30 % of the 64x32 search's wall time
// (tools/probes/bnb_profile.py).  Decision order and tie-breaks are the Python restatement's
// (tests/test_round_native.py compares the two leaf for leaf).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <numeric>
#include <vector>

#include "../../include/neptune_lp.h"

namespace {

// greedy first-fit of the candidates ks (flat (f, j), ascending) into the node memories in decreasing `key`
// order (ties: lower index first): every destination whose candidates all fit takes them all; the
// candidates of the others are walked by (destination, key desc, index)
void open_in_order(int N, const std::vector<int> &ks, const std::vector<double> &key, const double *fmem,
                   const std::vector<double> &room, std::vector<double> &used, std::vector<double> &c,
                   std::vector<double> &tot) {
  if (ks.empty()) return;
  std::fill(tot.begin(), tot.end(), 0.0);
  for (int k : ks) tot[k % N] += fmem[k / N];
  std::vector<char> fit(N, 0);
  for (int j = 0; j < N; ++j) fit[j] = tot[j] <= room[j] - used[j];
  std::vector<int> rest;
  for (size_t t = 0; t < ks.size(); ++t) {
    const int k = ks[t];
    if (fit[k % N]) c[k] = 1.0;
    else rest.push_back((int)t);
  }
  for (int j = 0; j < N; ++j)
    if (fit[j] && tot[j] > 0) used[j] += tot[j];
  if (rest.empty()) return;
  std::stable_sort(rest.begin(), rest.end(), [&](int a, int b) {
    const int ja = ks[a] % N, jb = ks[b] % N;
    if (ja != jb) return ja < jb;
    if (key[a] != key[b]) return key[a] > key[b];
    return ks[a] < ks[b];
  });
  for (int t : rest) {
    const int k = ks[t], j = k % N;
    const double mq = fmem[k / N];
    if (used[j] + mq <= room[j]) {
      c[k] = 1.0;
      used[j] += mq;
    }
  }
}

// the part of a rounding every mode shares: c from the node's fixings, the node memories they use, the closed
// placements, and the LP's near-integral placements opened (largest c first).  0: the fixings alone overfill a node
struct RoundPrefix {
  std::vector<double> c, used, room, tot;
  std::vector<char> closed;
};

int round_prefix(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const double *zc, const double *fn_mem,
                 const double *node_mem, RoundPrefix &r) {
  const size_t FN = (size_t)F * N;
  r.c.assign(FN, 0.0);
  r.used.assign(N, 0.0);
  r.room.resize(N);
  r.tot.resize(N);
  for (size_t k = 0; k < FN; ++k) r.c[k] = c_fix[k] > 0.5 ? 1.0 : 0.0;
  for (int j = 0; j < N; ++j) r.room[j] = node_mem[j] + 1e-9;
  for (int f = 0; f < F; ++f)
    for (int j = 0; j < N; ++j) r.used[j] += fn_mem[f] * r.c[(size_t)f * N + j];
  for (int j = 0; j < N; ++j)
    if (r.used[j] > r.room[j]) return 0;
  r.closed.resize(FN);
  for (size_t k = 0; k < FN; ++k) r.closed[k] = c_fix[k] >= 0 || (n_fix && n_fix[k % N] == 0.0);
  // the LP's near-integral placements first, largest c first
  std::vector<int> ks;
  std::vector<double> key;
  for (size_t k = 0; k < FN; ++k)
    if (!r.closed[k] && (zc ? zc[k] : 0.0) >= 0.5) { ks.push_back((int)k); key.push_back(zc[k]); }
  open_in_order(N, ks, key, fn_mem, r.room, r.used, r.c, r.tot);
  return 1;
}

// one mode from the shared prefix (r is this mode's copy): by flow above the threshold, then a destination for every
// function left without one, then n
int round_finish(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const float *flow, const double *zc,
                 const double *fn_mem, int32_t by_flow, double flow_threshold, RoundPrefix &r, double *c_out,
                 double *n_out) {
  const double NINF = -std::numeric_limits<double>::infinity();
  const size_t FN = (size_t)F * N;
  std::vector<double> &c = r.c, &used = r.used, &room = r.room, &tot = r.tot;
  const std::vector<char> &closed = r.closed;
  auto zcv = [&](size_t k) { return zc ? zc[k] : 0.0; };
  if (by_flow) {
    std::vector<int> ks;
    std::vector<double> key;
    for (size_t k = 0; k < FN; ++k)
      if (!closed[k] && c[k] < 0.5 && (double)flow[k] > flow_threshold) { ks.push_back((int)k); key.push_back(flow[k]); }
    open_in_order(N, ks, key, fn_mem, room, used, c, tot);
  }
  // each function left without a destination: the open-able destination with the largest LP c, then flow
  // (lowest index on ties), or the next one in (c desc, flow desc, index) order that still has room; the
  // choices of the later functions do not see these openings' c (only their memory)
  std::vector<size_t> opened;
  for (int f = 0; f < F; ++f) {
    double cnt = 0.0;
    for (int j = 0; j < N; ++j) cnt += c[(size_t)f * N + j];
    if (cnt >= 1) continue;
    double top = NINF;
    for (int j = 0; j < N; ++j)
      if (!closed[(size_t)f * N + j]) top = std::max(top, zcv((size_t)f * N + j));
    if (top == NINF) return 0;
    int first = 0;
    double best = NINF;
    bool any = false;
    for (int j = 0; j < N; ++j) {
      const size_t k = (size_t)f * N + j;
      const double v = (closed[k] || zcv(k) < top) ? NINF : (double)flow[k];
      if (!any || v > best) { best = v; first = j; any = true; }
    }
    int j = first;
    if (used[j] + fn_mem[f] > room[j]) {
      std::vector<int> order(N);
      std::iota(order.begin(), order.end(), 0);
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        const double za = zcv((size_t)f * N + a), zb = zcv((size_t)f * N + b);
        if (za != zb) return za > zb;
        return (double)flow[(size_t)f * N + a] > (double)flow[(size_t)f * N + b];
      });
      j = -1;
      for (int jj : order)
        if (!closed[(size_t)f * N + jj] && used[jj] + fn_mem[f] <= room[jj]) { j = jj; break; }
      if (j < 0) return 0;
    }
    opened.push_back((size_t)f * N + j);
    used[j] += fn_mem[f];
  }
  for (size_t k : opened) c[k] = 1.0;
  if (n_fix) {
    std::vector<double> nv(N, 0.0);
    for (int j = 0; j < N; ++j) {
      double s = 0.0;
      for (int f = 0; f < F; ++f) s += c[(size_t)f * N + j];
      nv[j] = s >= 1 ? 1.0 : 0.0;
    }
    std::vector<int> by_mem(F);
    std::iota(by_mem.begin(), by_mem.end(), 0);
    std::stable_sort(by_mem.begin(), by_mem.end(), [&](int a, int b) { return fn_mem[a] < fn_mem[b]; });
    for (int j = 0; j < N; ++j) {
      if (!(n_fix[j] == 1.0 && nv[j] == 0.0)) continue;
      int pick = -1;
      for (int f : by_mem)
        if (c_fix[(size_t)f * N + j] < 0 && used[j] + fn_mem[f] <= room[j]) { pick = f; break; }
      if (pick < 0) return 0;
      c[(size_t)pick * N + j] = 1.0;
      used[j] += fn_mem[pick];
      nv[j] = 1.0;
    }
    for (int j = 0; j < N; ++j)
      if (n_fix[j] == 0.0 && nv[j] == 1.0) return 0;
    if (n_out) std::copy(nv.begin(), nv.end(), n_out);
  }
  std::copy(c.begin(), c.end(), c_out);
  return 1;
}

}  // namespace

extern "C" int nep_round_leaf(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const float *flow,
                              const double *zc, const double *fn_mem, const double *node_mem, int32_t by_flow,
                              double flow_threshold, double *c_out, double *n_out) {
  if (F <= 0 || N <= 0 || !c_fix || !flow || !fn_mem || !node_mem || !c_out) return NEP_ERR_ARG;
  RoundPrefix r;
  if (!round_prefix(F, N, c_fix, n_fix, zc, fn_mem, node_mem, r)) return 0;
  return round_finish(F, N, c_fix, n_fix, flow, zc, fn_mem, by_flow, flow_threshold, r, c_out, n_out);
}

extern "C" int nep_round_leaves(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const float *flow,
                                const double *zc, const double *fn_mem, const double *node_mem, int32_t modes,
                                const int32_t *by_flow, const double *flow_threshold, double *c_out, double *n_out,
                                int32_t *found) {
  if (modes < 0 || (modes > 0 && (!by_flow || !flow_threshold || !c_out || !found))) return NEP_ERR_ARG;
  if (modes == 0) return NEP_OK;
  if (F <= 0 || N <= 0 || !c_fix || !flow || !fn_mem || !node_mem) return NEP_ERR_ARG;
  // the modes share the prefix (fixings, near-integral placements): computed once, copied per mode
  RoundPrefix pre, r;
  const int ok = round_prefix(F, N, c_fix, n_fix, zc, fn_mem, node_mem, pre);
  for (int k = 0; k < modes; ++k) {
    found[k] = 0;
    if (!ok) continue;
    r = pre;
    found[k] = round_finish(F, N, c_fix, n_fix, flow, zc, fn_mem, by_flow[k], flow_threshold[k], r,
                            c_out + (size_t)k * F * N, n_out ? n_out + (size_t)k * N : nullptr);
  }
  return NEP_OK;
}
