/*
 * neptune_lp.h — C ABI of the MI355X (gfx950) batched LP-relaxation engine for NEPTUNE's
 * node x function placement/routing MIP.
 *
 * What this replaces.  The reference hands the whole MIP to OR-Tools/SCIP through pywraplp:
 *   core/solvers/solver.py:7      pywraplp.Solver.CreateSolver('SCIP')        -> nep_model_create
 *   core/solvers/solver.py:15-20  load_data -> init_vars / init_constraints   -> nep_model_desc
 *   core/solvers/solver.py:35-40  init_objective(); Solver.Solve(); status == OPTIMAL
 *                                 (SCIP solves one LP relaxation per B&B node) -> nep_lp_solve_batch
 *                                                                               (nep_lp_submit/advance)
 *   core/solvers/solver.py:45-46  score() = Objective().Value()               -> obj / primal_obj
 *   neptune/utils/output.py:5-21  x[i,f,j].solution_value(), c[f,j], n[j]     -> nep_lp_get_solution
 * The model rows/columns are exactly those of neptune/utils/variables.py, constraints_step1.py,
 * constraints_step2.py and objectives.py (see DESIGN.md §2 for the row-by-row map).
 *
 * Conventions.  Plain pointers and sizes only.  Every call returns NEP_OK (0) on success or a
 * negative NEP_ERR_*; nep_last_error() gives a thread-local message.  Host arrays are read during
 * the call only.  The library owns all device workspaces; one model serves `max_batch` LP slots
 * (B&B nodes) that can be warm-started from each other.  A model's device work runs on its iteration
 * stream (the caller's or its own) and one auxiliary stream of the highest priority (slot reads, warm-start
 * copies, submits), ordered by events: a slot iterates only after its submit's initialisation; the HIP
 * context is created on first use (safe after fork()).
 *
 * Integer-variable vector ("z_int"), in the reference's variable-creation order minus x:
 *   step 1: c[F*N] (f-major), then n[N] (MinUtilization / MinDelayAndUtilization only)
 *   step 2: c[F*N], moved_from[F*N], moved_to[F*N], allocated, deallocated, then n[N] (MU / MDU)
 */
#ifndef NEPTUNE_LP_H
#define NEPTUNE_LP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NEP_API_VERSION 12

/* variants: neptune.py:41-66 (NeptuneMinDelay / MinUtilization / MinDelayAndUtilization) */
enum { NEP_MIN_DELAY = 0, NEP_MIN_UTILIZATION = 1, NEP_MIN_DELAY_AND_UTILIZATION = 2 };
/* steps: neptune_step1.py (step 1), neptune_step2.py mode="delete" / "create" */
enum { NEP_STEP1 = 1, NEP_STEP2_DELETE = 2, NEP_STEP2_CREATE = 3 };
/* API 7, nep_model_desc.relaxation: which LP the model iterates.
 *   NEP_RELAX_REFERENCE  the reference's own LP relaxation (constraints_step1.py / constraints_step2.py rows
 *                        as built, big-M pairs included): the LP SCIP solves at a B&B node
 *   NEP_RELAX_FACILITY   step 1 (MinUtilization / MinDelayAndUtilization) only: a STRENGTHENED relaxation
 *                        for branch-and-bound bounds: x[i,f,j] <= c[f,j] for every routing
 *                        row and c[f,j] <= n[j] (valid for every integral placement: constraints_step1.py:5-15,
 *                        :69-78 with c, n binary) replace the big-M pairs C1/C2 and C6/C7, which they imply
 *                        for integral c, n (C2 and C7, the eps floors, are relaxed); the capacity rows take n on
 *                        their right-hand side, C3 sum_f mem_f c[f,j] <= Mem_j n[j] and C5 CPU_j <= cores_j n[j]
 *                        (constraints_step1.py:18-23, :57-65: a closed node has neither).  Same variables, z_int
 *                        and objective; C4 and C8 kept.  Its bound is valid for the MIP, not equal to the
 *                        reference LP's */
enum { NEP_RELAX_REFERENCE = 0, NEP_RELAX_FACILITY = 1 };

enum { NEP_OK = 0, NEP_ERR_ARG = -1, NEP_ERR_HIP = -2, NEP_ERR_NOMEM = -3, NEP_ERR_STATE = -4 };

/* per-LP status */
enum {
  NEP_LP_OPTIMAL = 0,          /* certified: gap(primal obj, Lagrangian bound) and residuals <= tol */
  NEP_LP_ITERATION_LIMIT = 1,  /* obj still holds a VALID lower bound (Lagrangian) */
  NEP_LP_INFEASIBLE = 2,       /* proven by presolve (empty routing row, crossed bounds, row activity) */
  NEP_LP_CUTOFF = 3,           /* Lagrangian bound exceeded opts.cutoff: node can be pruned */
  NEP_LP_NUMERICAL = 4,
  NEP_LP_BOUND = 5             /* API 6, opts.bound_res > 0 only: the bound has converged (within gap_tol of
                                  the repaired point's objective, whose residual is <= bound_res) but the
                                  point is not certified feasible at tol; obj = the VALID Lagrangian bound.
                                  For B&B nodes that branch on the bound (not incumbents) */
};

typedef struct {
  int32_t n_nodes;             /* N */
  int32_t n_functions;         /* F */
  int32_t variant;             /* NEP_MIN_* */
  int32_t step;                /* NEP_STEP1 / NEP_STEP2_DELETE / NEP_STEP2_CREATE */
  double alpha;                /* neptune_step1.py:68 (default 0.5) */
  double soften_step1_sol;     /* neptune_step2.py:6 (default 1.3) */
  double max_score;            /* step 2: step-1 objective (neptune.py:22) */
  double prev_network_delay;   /* step 2 MinDelay: sum D[i,j] W[f,i] prev_x[i,f,j] (constraints_step2.py:66-68) */
  double big_m;                /* constraints_step1.py:1 (1e6) */
  double epsilon;              /* constraints_step1.py:2 (1e-6) */
  const double *delay;         /* [N*N] node_delay_matrix D[i][j] */
  const double *workload;      /* [F*N] workload_matrix W[f][i] (already * workload_coeff) */
  const double *core_per_req;  /* [F*N] core_per_req_matrix cpr[f][j] */
  const double *function_memory; /* [F] */
  const double *node_memory;   /* [N] */
  const double *node_cores;    /* [N] */
  const double *node_cost;     /* [N] (input_to_data.py:186: 5) */
  double node_budget;          /* (input_to_data.py:187: 300) */
  const double *max_delay;     /* [F] max_delay_matrix (input_to_data.py:136: 1000) */
  const double *old_allocations; /* [F*N] step 2 only (0/1) */
  int32_t relaxation;          /* API 7: NEP_RELAX_REFERENCE (0) or NEP_RELAX_FACILITY */
  int32_t device_inputs;       /* API 9: 1 = every array above is DEVICE memory (e.g. the data_ptr() of contiguous
                                  float64 PyTorch-ROCm tensors on the model's GPU); nep_model_create reads the
                                  O(F N + N^2) instance from there and builds the model (scaling on the host, the
                                  step size on the device).  0 = host arrays (nep_debug_* take host arrays only) */
} nep_model_desc;

typedef struct {
  double tol;                  /* certified relative tolerance (default 1e-7) */
  double cutoff;               /* stop when the Lagrangian bound exceeds this (default +inf) */
  int64_t max_iters;           /* default 200000 */
  int32_t check_every;         /* PDHG iterations between certificate checks (default 64) */
  int32_t warm_start;          /* 1: continue from the slot's current state (after nep_lp_copy_state) */
  double warm_omega_floor;     /* warm starts: the primal weight stays >= this x the parent's
                                  (0: default 2; < 0: no floor) */
  double gap_tol;              /* API 5: certified objective gap (relative, as tol); 0: = tol.  A tighter
                                  gap for an LP whose state warm-starts others (a B&B root) */
  double warm_omega_cap;       /* API 5: warm starts: the primal weight stays <= this x the parent's
                                  (0: default 4; < 0: no cap).  DESIGN.md §4 "Warm starts" */
  double polish_after;         /* API 5: primal feasibility polishing may start after this many
                                  iterations (0: default — 256 for warm starts, never for cold starts;
                                  < 0: never).  DESIGN.md §4 "Polishing" */
  double bound_res;            /* API 6: > 0: an LP whose bound has converged (gap <= gap_tol) while its
                                  repaired point's residual is within bound_res stops with NEP_LP_BOUND
                                  (0: never; a B&B sets it on branching nodes, never on leaves) */
} nep_lp_opts;

typedef struct {
  int32_t n_int;               /* length of z_int */
  int32_t n_rows;              /* R: routing rows after exact zero-workload source aggregation */
  int32_t n_tiles;             /* x-pass workgroups per LP (one per function) */
  int32_t max_batch;
  int64_t x_entries;           /* R*N per LP */
  int64_t bytes_per_iter;      /* algorithmic HBM bytes of one PDHG iteration of one LP */
  double step_size;            /* eta = 0.95 / ||K||_2 (scaled) */
  double primal_weight0;       /* API 10: the cold start's PDHG primal weight omega0 = ||c~|| / ||b~|| (scaled) */
} nep_model_info;

typedef struct {
  int64_t x_pass_launches;     /* launches of the fused routing-row kernel */
  double x_pass_ms;            /* summed HIP-event duration of the sampled x-pass launches */
  int64_t x_pass_sampled;      /* number of sampled launches in x_pass_ms */
  int64_t x_pass_lp_iters;     /* LP-iterations carried by the sampled launches */
  double solve_ms;             /* wall time inside nep_lp_solve_batch / nep_lp_advance (device-synchronised) */
  int64_t lp_iterations;       /* PDHG iterations summed over LPs */
} nep_stats;

int nep_model_create(const nep_model_desc *desc, int32_t max_batch, void *hip_stream, void **out_model);
void nep_model_destroy(void *model);
int nep_model_get_info(void *model, nep_model_info *info);

/* Solve B node LPs in slots[0..B-1] to completion.  lb_int/ub_int: host [B][n_int] bounds on z_int
 * (branching fixings; pass NULL for the root bounds).  Outputs (host, length B): obj = certified LP
 * value (Lagrangian lower bound), primal_obj = objective of the primal iterate, status, iters.
 * Equivalent to nep_lp_submit + nep_lp_advance until no slot iterates. */
int nep_lp_solve_batch(void *model, int32_t B, const int32_t *slots, const double *lb_int, const double *ub_int,
                       const nep_lp_opts *opts, double *obj, double *primal_obj, int32_t *status, int64_t *iters);

/* Streaming form, for a branch-and-bound that keeps every slot busy.
 * nep_lp_submit: start n node LPs in free slots (host presolve, then the slot's initialisation on
 *   the device).  status[b] = NEP_LP_INFEASIBLE when presolve proves node b infeasible (it does not
 *   iterate), NEP_LP_ITERATION_LIMIT when it starts iterating.  max_iters, warm_start and
 *   warm_omega_floor apply to the LPs of this call; tol and cutoff (the last submit's) to every LP
 *   in flight; check_every cannot change while any slot iterates.
 * nep_lp_advance: run blocks of check_every PDHG iterations on every iterating slot until at least
 *   min_done of them finished (min_done <= 0: exactly one block).  The finished slots and their
 *   results go to the first *n_done entries of the outputs (each sized max_batch).
 * nep_lp_active: number of iterating slots. */
int nep_lp_submit(void *model, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                  const nep_lp_opts *opts, int32_t *status);
/* API 12: nep_lp_submit with a per-LP iteration budget and bound stop (max_iters[b] / bound_res[b] for node
 * b; a NULL array takes the opts' value, an entry <= 0 opts->max_iters / no bound stop), so a
 * branch-and-bound starts its strong-branching probes, children and re-solves in one submit group. */
int nep_lp_submit_ex(void *model, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                     const nep_lp_opts *opts, const int64_t *max_iters, const double *bound_res, int32_t *status);
int nep_lp_advance(void *model, int32_t min_done, int32_t *n_done, int32_t *done_slots, double *obj,
                   double *primal_obj, int32_t *status, int64_t *iters);
int nep_lp_active(void *model);

/* z_int (host, n_int) and optionally the dense routing x[i][f][j] (host float, N*F*N) of a slot.  For a
 * certified slot (NEP_LP_OPTIMAL) z_int is the certificate's repaired point — the primal solution
 * whose objective primal_obj is and whose rows the certificate checked — else the PDHG iterate. */
int nep_lp_get_solution(void *model, int32_t slot, double *z_int, float *x_dense);
/* API 8: z_int of n finished slots at once (z_out [n][n_int], each as nep_lp_get_solution's): one device
 * round trip for all the branching nodes an advance returned. */
int nep_lp_get_solutions(void *model, int32_t n, const int32_t *slots, double *z_out);
/* API 12: nep_lp_get_flows and nep_lp_get_solutions of the same n slots in one device round trip (one wait) */
int nep_lp_get_flows_solutions(void *model, int32_t n, const int32_t *slots, float *flows, double *z_out);
/* aggregated routing rows (host float, R*N) and the row map (row_f, row_src; src = -1: pooled
 * zero-workload sources of function f, each routed identically). */
int nep_lp_get_rows(void *model, int32_t slot, float *xbar, int32_t *row_f, int32_t *row_src);
/* copy a slot's primal/dual state to another (not iterating) slot: warm start of a child node */
int nep_lp_copy_state(void *model, int32_t src_slot, int32_t dst_slot);
/* API 12: n such copies with the result of n nep_lp_copy_state calls in order, in as few launches as their overlaps
 * allow (a B&B submit's warm-start copies: usually one) */
int nep_lp_copy_states(void *model, int32_t n, const int32_t *src_slots, const int32_t *dst_slots);

/* tol / cutoff of every LP in flight, effective from the next iteration block (a B&B lowers the
 * cutoff to each new incumbent without resubmitting). */
int nep_lp_set_params(void *model, double tol, double cutoff);

/* API 10: the primal-weight band of warm starts.  omega_ref > 0: a warm-started LP takes its weight in
 * [warm_omega_floor, warm_omega_cap] x omega_ref (its parent's weight clamped into that band) instead of
 * relative to its parent's final weight, which ratchets up along a lineage of warm starts (DESIGN.md §4
 * "Warm-start primal weight"); 0 restores the parent-relative band.  Applies to later submits. */
int nep_lp_set_reference_weight(void *model, double omega_ref);

/* flow[b][f][j] = sum_i x[i,f,j] of finished slots (host float, n x F x N), computed on the device:
 * the branch-and-bound's branching / rounding input (replaces copying the R x N routing rows). */
int nep_lp_get_flows(void *model, int32_t n, const int32_t *slots, float *flows);
/* API 6: the same flows and, in wflows, their part carried by workload sources only (W[f,i] > 0: the
 * pooled zero-workload row excluded — its mass is free to go to any open placement); the B&B's
 * rounding opens placements for workload, not for that free mass. */
int nep_lp_get_flows_split(void *model, int32_t n, const int32_t *slots, float *flows, float *wflows);

/* Wire format on the device (neptune/utils/output.py:23-39).  Routing entries of the aggregated rows
 * with x > threshold (0.001), value rounded as np.round(x, 3) when round3; allocation entries c[f,j] >
 * threshold.  Row-major order.  Call with capacity 0 (or too small) to get *n_entries only; the row
 * map of nep_lp_get_rows expands a pooled row (src = -1) to all zero-workload sources of its f. */
int nep_lp_routing_entries(void *model, int32_t slot, double threshold, int32_t round3, int64_t capacity,
                           int64_t *n_entries, int32_t *row, int32_t *dst, double *val);
int nep_lp_allocation_entries(void *model, int32_t slot, double threshold, int64_t capacity, int64_t *n_entries,
                              int32_t *fn, int32_t *dst);

/* The reference's offline scorers and feasibility checkers on a slot's solution, on the device
 * (efttc/utils/objectives.py:23-98, efttc/utils/constraints_step1.py:5-133; booleans are the
 * reference's truthiness, value != 0).  out[NEP_SC_COUNT]: */
enum {
  NEP_SC_NETWORK_DELAY = 0,   /* score_minimize_network_delay: sum W[f,i] D[i,j] x[i,f,j] */
  NEP_SC_NODES_USED = 1,      /* score_minimize_node_utilization: #{j : n[j] != 0} */
  NEP_SC_NODE_COST = 2,       /* sum n[j] cost[j] (constrain_budget) */
  NEP_SC_BAD_C_X = 3,         /* constrain_c_according_to_x violations (f, j) */
  NEP_SC_BAD_MEMORY = 4,      /* constrain_memory_usage violations (nodes) */
  NEP_SC_BAD_HANDLE = 5,      /* constrain_handle_all_requests: (i, f) with |sum_j x - 1| >= 0.1 */
  NEP_SC_BAD_CPU = 6,         /* constrain_CPU_usage violations (nodes, + 1e-6) */
  NEP_SC_BAD_N_C = 7,         /* constrain_n_according_to_c violations (nodes) */
  NEP_SC_BAD_BUDGET = 8,      /* constrain_budget (0 / 1) */
  NEP_SC_HANDLE_MAXDEV = 9,   /* max |sum_j x - 1| */
  NEP_SC_CPU_MAXEXCESS = 10,  /* max (CPU use - cores, 0) */
  NEP_SC_COUNT = 11
};
int nep_lp_score_check(void *model, int32_t slot, double *out);

int nep_get_stats(void *model, nep_stats *stats);

/* diagnostics: out16 = {primal obj, Lagrangian, best Lagrangian, primal residual, gap, omega, tau,
 * sigma, eta, iterations, iterations since restart, status, active, fpr at restart, last fpr, ||K||} */
int nep_lp_get_diag(void *model, int32_t slot, double *out16);
/* device state of a slot (any pointer may be NULL): duals [n_dual], row activities [n_dual],
 * packed f32 duals of the x pass [F*NP+NP+4], node bounds [n_int] */
int nep_debug_state(void *model, int32_t slot, double *y, double *kz, float *kty, double *lb, double *ub);
/* API 12: per routing row of a slot (length R), the nonzeros its Halpern anchor is held with (17 = dense) and, on a
 * facility-relaxation model, the nonzeros of its x <= c duals (counted on the host) */
int nep_debug_sparse_rows(void *model, int32_t slot, int32_t *anchor_cnt, float *lambda_nnz);
/* host-only model build (no device work): step size, scalings, row norms, dims = {R, F, n_int,
 * n_dual}.  Lets the CPU test-suite check the model build without a GPU. */
int nep_debug_build(const nep_model_desc *desc, double *eta, double *rho, double *gam, double *rownorm,
                    int32_t *dims);
/* host-only node presolve of n nodes (lb_int/ub_int as for nep_lp_submit), evaluated twice: from
 * scratch and as the sparse change of the model's base box that nep_lp_submit uses.  ok_* [n]:
 * 1 = feasible; box_* [n][2][n_int] (may be NULL): the resulting node bounds (lb then ub). */
int nep_debug_presolve(const nep_model_desc *desc, int32_t n, const double *lb_int, const double *ub_int,
                       int32_t *ok_full, int32_t *ok_node, double *box_full, double *box_node);
void nep_reset_stats(void *model);

/* API 8: the routing state (x and its projection thresholds) of a finished slot of ANOTHER model of the same
 * instance and row layout (e.g. a NEP_RELAX_FACILITY branching node) copied into a finished slot of this one —
 * a leaf's warm start from its branching node's routing; the slot's other state (small variables, duals) is
 * left as it is (typically the root's, nep_lp_copy_state); the next submit with warm_start iterates from it.
 * NEP_ERR_ARG when the row layouts differ.  Replaces SCIP's LP warm start across its own node LPs. */
int nep_lp_copy_routing(void *dst_model, int32_t dst_slot, void *src_model, int32_t src_slot);

/* API 8: branch-and-bound rounding heuristic (host only, no model; core/engine/bnb.py): one branching
 * node's LP -> a leaf fixing every c (and n).  c_fix [F*N] / n_fix [N] (n_fix NULL: no n): -1 free, 0 / 1
 * fixed by the node; flow [F*N] the node's flows, zc [F*N] its c (NULL: 0).  Fixed-open c first, then the free
 * c with zc >= 1/2 (largest first), then (by_flow) the free (f, j) with flow > flow_threshold (largest
 * first), each while node j's memory has room (constraints_step1.py:18-23); a function left without a
 * destination gets the one with the largest c, then flow; n = any c; a node fixed open gets its smallest
 * fitting function.  Returns 1 and fills c_out [F*N] (n_out [N]) with the leaf, 0 when the node has none,
 * < 0 on a bad argument.  Replaces the reference's nothing: SCIP's own primal heuristics run inside
 * Solve() (core/solvers/solver.py:37). */
int nep_round_leaf(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const float *flow, const double *zc,
                   const double *fn_mem, const double *node_mem, int32_t by_flow, double flow_threshold, double *c_out,
                   double *n_out);
/* API 8: nep_round_leaf for `modes` (by_flow[k], flow_threshold[k]) pairs of one node in one call: c_out
 * [modes][F*N], n_out [modes][N] (NULL without n), found[k] = 1 / 0 (< 0 returned on a bad argument). */
int nep_round_leaves(int32_t F, int32_t N, const double *c_fix, const double *n_fix, const float *flow, const double *zc,
                     const double *fn_mem, const double *node_mem, int32_t modes, const int32_t *by_flow,
                     const double *flow_threshold, double *c_out, double *n_out, int32_t *found);

/* API 11: the branch-and-bound's tree search, native (csrc/nep_bnb.cpp; core/engine/bnb.py delegates its
 * single-rank step-1 search here, DESIGN.md §7 "Native tree search").  Replaces the host loop of
 * BranchAndBound.solve (core/engine/bnb.py) — the tree SCIP searches inside Solver.Solve()
 * (core/solvers/solver.py:35-40): best-first open nodes, rounding leaves, retries of uncertified leaves,
 * warm starts from the parent's slot or the root's state, one submit / advance stream per model (the leaf
 * model = the reference LP; the optional bound model = the facility relaxation), prune / branch / round per
 * finished LP.  The tree drives the models through this header's nep_lp_* calls only. */
typedef struct {
  int32_t c0, c1, n0, n1, n_int;   /* integer layout: c = z_int[c0:c1] (F x N), n = z_int[n0:n1] (n0 < 0: none) */
  int32_t F, N;
  int32_t warm;                    /* warm starts (reserves the leaf model's last two slots: root / incumbent state) */
  int32_t batch, batch_b;          /* LPs in flight per model (leaf, bound); further free slots keep finished states */
  int32_t check_every, root_check_every;
  int32_t unit_flow_leaves;        /* a third rounding mode: (f, j) carrying a unit of flow */
  int32_t objective_integral;      /* every integral point's objective is integral: prune at incumbent - 1 */
  int32_t primal_at_root;          /* nep_bnb_run returns NEP_BNB_ROOT once the root branching node finished */
  double tol, gap, bound_gap;      /* LP tolerance, relative MIP gap, the bound model's gap_tol */
  int64_t max_iters, node_max_iters, root_max_iters;
  double node_bound_res, retry_res, flow_tol;
  double upper_bound;              /* a-priori cutoff (+inf: none) */
  int64_t node_limit;
  double time_limit;               /* seconds (<= 0: none) */
  int32_t world, rank;             /* API 12: the sharded search (world > 1: NEP_BNB_SYNC once per loop) */
  int32_t branching;               /* API 12: 0 n by inflow, then c by flow; 1 pseudo-cost (product score);
                                      2 reliability branching: pseudo-costs, strong-branching probes while unreliable */
  int32_t strong_cands, strong_rel;  /* branching 2: candidates scored, observations per direction to be reliable */
  int32_t reserved_p;
  int64_t strong_iters;            /* branching 2: iteration budget of a probe LP */
  double objective_unit;           /* with objective_integral: the objective's integral unit (<= 0: 1) — e.g. alpha / N
                                      for MinDelayAndUtilization without workload, whose objective is alpha / N sum n */
} nep_bnb_params;

typedef struct {
  int64_t nodes, leaves, lps, certified, lp_iterations, unresolved, drained;
  int64_t lp_status[7];            /* certified, bound, limit, infeasible, cutoff, numerical, presolve-infeasible */
  int64_t lp_status_kind[4][7];    /* per node kind: node, leaf, retry, refroot */
  int64_t advance_calls, inflight_sum, lp_incumbents, heuristic_incumbents, n_lp_iters;
  double advance_seconds, finish_seconds, submit_seconds, drain_seconds, root_seconds;
  double bound, incumbent;         /* at the end: best proven bound, incumbent value (+inf: none) */
  int32_t incumbent_source;        /* 0 none, 1 a certified leaf LP, 2 nep_bnb_set_incumbent */
  int32_t incumbent_slot;          /* leaf-model slot holding the incumbent LP's state (source 1) */
  int32_t limit_hit, any_unresolved, unresolved_below;
  int32_t stalled;                 /* API 12: ended because open nodes could never get a slot (reported as a limit) */
  uint32_t split_hash;             /* sharded: crc32 of the frontier every rank dealt (bnb.py _frontier_hash) */
  int32_t reserved_;
  int64_t presplit_nodes, presplit_lps, presplit_certified;   /* sharded: counts when the frontier was dealt */
  int64_t rebalanced, sync_calls;  /* sharded: open nodes imported from other ranks; collectives answered */
  double agreed_incumbent;         /* min(this rank's incumbent, the ranks' agreed one) */
  int64_t strong_nodes, strong_lps, strong_iterations, strong_decided;   /* branching 2: nodes that probed, probes */
} nep_bnb_stats;

#define NEP_BNB_DONE 0   /* the search ended (no open node, or a stop): stats / incumbent are final */
#define NEP_BNB_ROOT 1   /* the root branching node finished: nep_bnb_event_data, then nep_bnb_add_leaf(where = 1) /
                            nep_bnb_set_incumbent for the caller's primal heuristic, then nep_bnb_run again */
#define NEP_BNB_INCUMBENT 2   /* (nep_bnb_set_step2 with incumbent_events) a new LP incumbent: nep_bnb_incumbent_event,
                                 then nep_bnb_add_leaf(where = 2) for each neighbour leaf, then nep_bnb_run again */
#define NEP_BNB_SYNC 3   /* (world > 1) the loop's collective is due: nep_bnb_sync_get, the caller's all-reduce over the
                            ranks (incumbent MIN, stop OR, open SUM; core/engine/comm.py agree), nep_bnb_sync_set,
                            optionally a rebalance (nep_bnb_export_nodes / nep_bnb_import_nodes), then nep_bnb_run */

/* API 12: the calls the tree makes on one model, with the model's integer vector length and slot count.
 * nep_bnb_create fills one from an engine handle (the nep_lp_* functions, ctx = the handle); a caller may pass its
 * own (the CPU suite: HiGHS node LPs behind ctypes callbacks).  Same contracts as the nep_lp_* functions. */
typedef struct {
  void *ctx;
  int32_t n_int, max_batch;
  int (*submit)(void *ctx, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                const nep_lp_opts *opts, int32_t *status);
  int (*advance)(void *ctx, int32_t min_done, int32_t *n_done, int32_t *done_slots, double *obj, double *primal_obj,
                 int32_t *status, int64_t *iters);
  int (*active)(void *ctx);
  int (*copy_state)(void *ctx, int32_t src_slot, int32_t dst_slot);
  int (*set_params)(void *ctx, double tol, double cutoff);
  int (*get_flows)(void *ctx, int32_t n, const int32_t *slots, float *flows);
  int (*get_solutions)(void *ctx, int32_t n, const int32_t *slots, double *z_out);
  int (*get_diag)(void *ctx, int32_t slot, double *out16);
  /* optional (NULL: one submit per budget / bound-stop group): nep_lp_submit_ex's contract */
  int (*submit_ex)(void *ctx, int32_t n, const int32_t *slots, const double *lb_int, const double *ub_int,
                   const nep_lp_opts *opts, const int64_t *max_iters, const double *bound_res, int32_t *status);
  /* optional (NULL: copy_state per pair): nep_lp_copy_states' contract */
  int (*copy_states)(void *ctx, int32_t n, const int32_t *src_slots, const int32_t *dst_slots);
  /* optional (NULL: get_flows, then get_solutions): nep_lp_get_flows_solutions' contract */
  int (*get_flows_solutions)(void *ctx, int32_t n, const int32_t *slots, float *flows, double *z_out);
} nep_bnb_engine;

/* NULL on a bad argument (nep_last_error says which): batch < 1, a layout outside n_int, no working slot left
 * after the reserved ones, world / rank out of range. */
void *nep_bnb_create(void *leaf_model, void *bound_model, const nep_bnb_params *params, const double *fn_mem,
                     const double *node_mem);
void *nep_bnb_create_engines(const nep_bnb_engine *leaf, const nep_bnb_engine *bound, const nep_bnb_params *params,
                             const double *fn_mem, const double *node_mem);
void nep_bnb_destroy(void *tree);
/* a leaf (a full c / n assignment, or any box): where = 0 a seed leaf queued when the root LP finishes;
 * where = 1 a leaf of the NEP_BNB_ROOT event's node, where = 2 a neighbour of the NEP_BNB_INCUMBENT event's
 * leaf, both at the front of the leaf queue */
int nep_bnb_add_leaf(void *tree, int32_t n, const int32_t *idx, const double *val, double bound, int32_t where);
/* step 2 (before the first nep_bnb_run): the closed-form integer bound of NeptuneStep2Base.integer_bound
 * (core/solvers/neptune/neptune_step.py; create != 0: create mode, node_cap: the most nodes an integral placement
 * opens, +inf: none; old_alloc [F*N]) on every node / leaf, and (incumbent_events) NEP_BNB_INCUMBENT events */
int nep_bnb_set_step2(void *tree, int32_t create, double node_cap, const double *old_alloc, int32_t incumbent_events);
int nep_bnb_incumbent_event(void *tree, int32_t *n_fix, int32_t *idx, double *val, double *value);
/* host only: that integer bound of one box (params: the layout fields), for the CPU suite */
int nep_bnb_debug_ibound(const nep_bnb_params *params, int32_t create, double node_cap, const double *old_alloc,
                         int32_t n, const int32_t *idx, const double *val, double *out);
/* an incumbent found outside the tree (a checked heuristic point): its value becomes the cutoff */
int nep_bnb_set_incumbent(void *tree, double value);
int nep_bnb_event_data(void *tree, double *z_int, float *flow);
int nep_bnb_run(void *tree, int32_t *event);
/* NEP_BNB_SYNC: out6 = {incumbent, stop, open + in-flight nodes, heap size, frontier dealt, collectives so far};
 * the caller answers with the agreed values (a lower incumbent becomes every model's cutoff at once) */
int nep_bnb_sync_get(void *tree, double *out6);
int nep_bnb_sync_set(void *tree, double incumbent, int32_t stop, int64_t open_total);
/* rebalance (bnb.py _rebalance): the k best-bound open nodes leave this rank's heap (lens[k]; meta[k][3] = bound,
 * depth, kind; idx / val concatenated, at most cap entries) / enter it (pruned against the incumbent; they start
 * from the model's root state) */
int nep_bnb_export_nodes(void *tree, int32_t k, int32_t cap, int32_t *lens, double *meta, int32_t *idx, double *val);
int nep_bnb_import_nodes(void *tree, int32_t k, const int32_t *lens, const double *meta, const int32_t *idx,
                         const double *val);
int nep_bnb_get_stats(void *tree, nep_bnb_stats *out);
int nep_bnb_get_lp_iters(void *tree, int64_t *out);
/* the LP incumbent's integer vector (n_int) and its leaf box (at most c1 - c0 + n1 - n0 entries: a leaf fixes every
 * c and n; *n_fix = -1: no LP incumbent) */
int nep_bnb_incumbent(void *tree, double *z_int, int32_t *n_fix, int32_t *idx, double *val);

const char *nep_last_error(void);
int nep_api_version(void);

#ifdef __cplusplus
}
#endif
#endif
