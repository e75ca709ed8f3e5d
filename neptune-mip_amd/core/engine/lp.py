"""ctypes binding of the MI355X LP engine (`include/neptune_lp.h`, lib/libneptune_lp.so).

This is the product path: there is no CPU fallback.  If the shared library is missing (not built)
or no GPU is visible, every call raises `EngineUnavailable` loudly.
"""
import ctypes
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NEPTUNE_LP_LIB",
                          os.path.normpath(os.path.join(_HERE, "..", "..", "lib", "libneptune_lp.so")))

MIN_DELAY, MIN_UTILIZATION, MIN_DELAY_AND_UTILIZATION = 0, 1, 2
STEP1, STEP2_DELETE, STEP2_CREATE = 1, 2, 3
LP_OPTIMAL, LP_ITERATION_LIMIT, LP_INFEASIBLE, LP_CUTOFF, LP_NUMERICAL, LP_BOUND = 0, 1, 2, 3, 4, 5
VARIANTS = {"MinDelay": MIN_DELAY, "MinUtilization": MIN_UTILIZATION,
            "MinDelayAndUtilization": MIN_DELAY_AND_UTILIZATION}
API_VERSION = 12
RELAX_REFERENCE, RELAX_FACILITY = 0, 1

_dp = ctypes.POINTER(ctypes.c_double)


class EngineUnavailable(RuntimeError):
    pass


class ModelDesc(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("n_functions", ctypes.c_int32), ("variant", ctypes.c_int32),
                ("step", ctypes.c_int32), ("alpha", ctypes.c_double), ("soften_step1_sol", ctypes.c_double),
                ("max_score", ctypes.c_double), ("prev_network_delay", ctypes.c_double),
                ("big_m", ctypes.c_double), ("epsilon", ctypes.c_double),
                ("delay", _dp), ("workload", _dp), ("core_per_req", _dp), ("function_memory", _dp),
                ("node_memory", _dp), ("node_cores", _dp), ("node_cost", _dp), ("node_budget", ctypes.c_double),
                ("max_delay", _dp), ("old_allocations", _dp), ("relaxation", ctypes.c_int32),
                ("device_inputs", ctypes.c_int32)]


class LpOpts(ctypes.Structure):
    _fields_ = [("tol", ctypes.c_double), ("cutoff", ctypes.c_double), ("max_iters", ctypes.c_int64),
                ("check_every", ctypes.c_int32), ("warm_start", ctypes.c_int32),
                ("warm_omega_floor", ctypes.c_double), ("gap_tol", ctypes.c_double),
                ("warm_omega_cap", ctypes.c_double),
                ("polish_after", ctypes.c_double), ("bound_res", ctypes.c_double)]


class ModelInfo(ctypes.Structure):
    _fields_ = [("n_int", ctypes.c_int32), ("n_rows", ctypes.c_int32), ("n_tiles", ctypes.c_int32),
                ("max_batch", ctypes.c_int32), ("x_entries", ctypes.c_int64), ("bytes_per_iter", ctypes.c_int64),
                ("step_size", ctypes.c_double), ("primal_weight0", ctypes.c_double)]


class Stats(ctypes.Structure):
    _fields_ = [("x_pass_launches", ctypes.c_int64), ("x_pass_ms", ctypes.c_double),
                ("x_pass_sampled", ctypes.c_int64), ("x_pass_lp_iters", ctypes.c_int64),
                ("solve_ms", ctypes.c_double), ("lp_iterations", ctypes.c_int64)]


class BnbParams(ctypes.Structure):
    _fields_ = [("c0", ctypes.c_int32), ("c1", ctypes.c_int32), ("n0", ctypes.c_int32), ("n1", ctypes.c_int32),
                ("n_int", ctypes.c_int32), ("F", ctypes.c_int32), ("N", ctypes.c_int32), ("warm", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("batch_b", ctypes.c_int32),
                ("check_every", ctypes.c_int32), ("root_check_every", ctypes.c_int32),
                ("unit_flow_leaves", ctypes.c_int32), ("objective_integral", ctypes.c_int32),
                ("primal_at_root", ctypes.c_int32), ("tol", ctypes.c_double), ("gap", ctypes.c_double),
                ("bound_gap", ctypes.c_double), ("max_iters", ctypes.c_int64), ("node_max_iters", ctypes.c_int64),
                ("root_max_iters", ctypes.c_int64), ("node_bound_res", ctypes.c_double),
                ("retry_res", ctypes.c_double), ("flow_tol", ctypes.c_double), ("upper_bound", ctypes.c_double),
                ("node_limit", ctypes.c_int64), ("time_limit", ctypes.c_double),
                ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("branching", ctypes.c_int32),
                ("strong_cands", ctypes.c_int32), ("strong_rel", ctypes.c_int32), ("reserved_p", ctypes.c_int32),
                ("strong_iters", ctypes.c_int64), ("objective_unit", ctypes.c_double)]


class BnbStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in ("nodes", "leaves", "lps", "certified", "lp_iterations", "unresolved",
                                              "drained")] + \
               [("lp_status", ctypes.c_int64 * 7), ("lp_status_kind", (ctypes.c_int64 * 7) * 4)] + \
               [(k, ctypes.c_int64) for k in ("advance_calls", "inflight_sum", "lp_incumbents", "heuristic_incumbents",
                                              "n_lp_iters")] + \
               [(k, ctypes.c_double) for k in ("advance_seconds", "finish_seconds", "submit_seconds", "drain_seconds",
                                               "root_seconds", "bound", "incumbent")] + \
               [(k, ctypes.c_int32) for k in ("incumbent_source", "incumbent_slot", "limit_hit", "any_unresolved",
                                              "unresolved_below", "stalled")] + \
               [("split_hash", ctypes.c_uint32), ("reserved_", ctypes.c_int32)] + \
               [(k, ctypes.c_int64) for k in ("presplit_nodes", "presplit_lps", "presplit_certified", "rebalanced",
                                              "sync_calls")] + \
               [("agreed_incumbent", ctypes.c_double)] + \
               [(k, ctypes.c_int64) for k in ("strong_nodes", "strong_lps", "strong_iterations", "strong_decided")]


# nep_bnb_engine (API 12): the calls the native tree makes on one model
_i32p, _i64p, _dblp = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)
_fltp = ctypes.POINTER(ctypes.c_float)
BNB_SUBMIT = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _dblp, _dblp,
                              ctypes.POINTER(LpOpts), _i32p)
BNB_ADVANCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _i32p, _dblp, _dblp, _i32p,
                               _i64p)
BNB_ACTIVE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
BNB_COPY = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32)
BNB_PARAMS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_double, ctypes.c_double)
BNB_FLOWS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _fltp)
BNB_SOLS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _dblp)
BNB_DIAG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _dblp)
BNB_COPIES = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _i32p)
BNB_FLOWS_SOLS = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _fltp, _dblp)
BNB_SUBMIT_EX = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, _i32p, _dblp, _dblp,
                                 ctypes.POINTER(LpOpts), _i64p, _dblp, _i32p)


class BnbEngine(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("n_int", ctypes.c_int32), ("max_batch", ctypes.c_int32),
                ("submit", BNB_SUBMIT), ("advance", BNB_ADVANCE), ("active", BNB_ACTIVE), ("copy_state", BNB_COPY),
                ("set_params", BNB_PARAMS), ("get_flows", BNB_FLOWS), ("get_solutions", BNB_SOLS),
                ("get_diag", BNB_DIAG), ("submit_ex", BNB_SUBMIT_EX), ("copy_states", BNB_COPIES),
                ("get_flows_solutions", BNB_FLOWS_SOLS)]


class PyBnbEngine:
    """A nep_bnb_engine call table over a Python model with LPModel's streaming interface (submit / advance /
    active / copy_state / set_params / flows / solutions / diag, n_int, max_batch): lets the native tree search
    (csrc/nep_bnb.cpp, nep_bnb_create_engines) drive node LPs that are not the engine's — the CPU suite runs it
    over HiGHS (tests/oracle_lp.py).  A Python exception inside a call ends the search with NEP_ERR_STATE and is
    kept in `error` (BranchAndBound re-raises it)."""

    def __init__(self, model, F, N, per_lp=True):
        self.model, self.F, self.N = model, int(F), int(N)
        self.n_int, self.max_batch = int(model.n_int), int(model.max_batch)
        self.error = None
        self.ex_calls = 0
        self.copies_calls = 0
        self.flows_sols_calls = 0
        ni, mb = self.n_int, self.max_batch
        A = np.ctypeslib.as_array

        def guard(fn):
            def call(*args):
                try:
                    fn(*args)
                    return 0
                except BaseException as e:      # (never unwind through the C frames)
                    self.error = e
                    return -4
            return call

        def submit(_, n, slots, lb, ub, opts, status):
            o = opts.contents
            st = model.submit(A(slots, (n,)).copy(), A(lb, (n, ni)).copy(), A(ub, (n, ni)).copy(), tol=o.tol,
                              cutoff=o.cutoff, max_iters=int(o.max_iters), check_every=int(o.check_every),
                              warm_start=bool(o.warm_start), bound_res=o.bound_res, gap_tol=o.gap_tol)
            A(status, (n,))[:] = np.asarray(st, np.int32)

        def submit_ex(_, n, slots, lb, ub, opts, mi, br, status):
            # per-LP budgets / bound stops: one model.submit per distinct (budget, bound stop), in first-seen order
            o = opts.contents
            sl, lbs, ubs = A(slots, (n,)).copy(), A(lb, (n, ni)).copy(), A(ub, (n, ni)).copy()
            mis = A(mi, (n,)).copy() if mi else np.full(n, o.max_iters, np.int64)
            brs = A(br, (n,)).copy() if br else np.full(n, o.bound_res)
            keys = list(dict.fromkeys(zip(mis.tolist(), brs.tolist())))
            out = A(status, (n,))
            for k_mi, k_br in keys:
                sel = np.flatnonzero((mis == k_mi) & (brs == k_br))
                st = model.submit(sl[sel], lbs[sel], ubs[sel], tol=o.tol, cutoff=o.cutoff,
                                  max_iters=int(k_mi) if k_mi > 0 else int(o.max_iters),
                                  check_every=int(o.check_every), warm_start=bool(o.warm_start),
                                  bound_res=max(float(k_br), 0.0), gap_tol=o.gap_tol)
                out[sel] = np.asarray(st, np.int32)
            self.ex_calls += 1

        def advance(_, min_done, n_done, slots, obj, pobj, status, iters):
            r = model.advance(int(min_done))
            k = len(r["slots"])
            n_done[0] = k
            if k:
                A(slots, (mb,))[:k] = r["slots"]
                A(obj, (mb,))[:k] = r["obj"]
                A(pobj, (mb,))[:k] = r["primal_obj"]
                A(status, (mb,))[:k] = r["status"]
                A(iters, (mb,))[:k] = r["iters"]

        def copy_state(_, src, dst):
            model.copy_state(int(src), int(dst))

        def copy_states(_, n, src, dst):
            # (the Python model copies pair by pair, in order: the contract of nep_lp_copy_states)
            for a, b in zip(A(src, (n,)).tolist(), A(dst, (n,)).tolist()):
                model.copy_state(int(a), int(b))
            self.copies_calls += 1

        def set_params(_, tol, cutoff):
            model.set_params(tol, cutoff)

        def flows(_, n, slots, out):
            A(out, (n * self.F * self.N,))[:] = np.asarray(model.flows(A(slots, (n,)).copy()), np.float32).ravel()

        def sols(_, n, slots, out):
            A(out, (n * ni,))[:] = np.asarray(model.solutions(A(slots, (n,)).copy()), np.float64).ravel()

        def flows_sols(_, n, slots, fout, zout):
            flows(_, n, slots, fout)
            sols(_, n, slots, zout)
            self.flows_sols_calls += 1

        def diag(_, slot, out):
            d = model.diag(int(slot))
            o = A(out, (16,))
            o[:] = 0.0
            o[3] = float(d.get("pres", 0.0))

        def active(_):
            try:
                return int(model.active())
            except BaseException as e:
                self.error = e
                return 0

        self.table = BnbEngine(None, ni, mb, BNB_SUBMIT(guard(submit)), BNB_ADVANCE(guard(advance)),
                               BNB_ACTIVE(active), BNB_COPY(guard(copy_state)), BNB_PARAMS(guard(set_params)),
                               BNB_FLOWS(guard(flows)), BNB_SOLS(guard(sols)), BNB_DIAG(guard(diag)),
                               BNB_SUBMIT_EX(guard(submit_ex)) if per_lp else BNB_SUBMIT_EX(),
                               BNB_COPIES(guard(copy_states)) if per_lp else BNB_COPIES(),
                               BNB_FLOWS_SOLS(guard(flows_sols)) if per_lp else BNB_FLOWS_SOLS())


# every entry point declared in include/neptune_lp.h
EXPORTS = ("nep_model_create", "nep_model_destroy", "nep_model_get_info", "nep_lp_solve_batch",
           "nep_lp_submit", "nep_lp_submit_ex", "nep_lp_advance", "nep_lp_active", "nep_lp_copy_states", "nep_lp_get_flows_solutions",
           "nep_lp_get_solution", "nep_lp_get_rows", "nep_lp_copy_state", "nep_get_stats", "nep_reset_stats",
           "nep_lp_get_flows_split",
           "nep_last_error", "nep_api_version", "nep_lp_get_diag", "nep_debug_build", "nep_debug_state",
           "nep_debug_presolve", "nep_debug_sparse_rows", "nep_lp_set_params", "nep_lp_get_flows", "nep_lp_routing_entries",
           "nep_lp_allocation_entries", "nep_lp_score_check", "nep_round_leaf", "nep_lp_copy_routing",
           "nep_lp_get_solutions", "nep_round_leaves", "nep_lp_set_reference_weight",
           "nep_bnb_create", "nep_bnb_destroy", "nep_bnb_add_leaf", "nep_bnb_set_incumbent", "nep_bnb_event_data",
           "nep_bnb_run", "nep_bnb_get_stats", "nep_bnb_get_lp_iters", "nep_bnb_incumbent", "nep_bnb_set_step2",
           "nep_bnb_incumbent_event", "nep_bnb_debug_ibound", "nep_bnb_create_engines", "nep_bnb_sync_get",
           "nep_bnb_sync_set", "nep_bnb_export_nodes", "nep_bnb_import_nodes")
SCORE_FIELDS = ("network_delay", "nodes_used", "node_cost", "bad_c_x", "bad_memory", "bad_handle", "bad_cpu",
                "bad_n_c", "bad_budget", "handle_maxdev", "cpu_maxexcess")

_lib = None


def _host_inputs():
    return os.environ.get("NEP_HOST_INPUTS", "0") not in ("", "0")


def load_library(path=None):
    """Load (once) and type the shared library.  Raises EngineUnavailable when absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise EngineUnavailable(f"MI355X LP engine not built: {p} missing (run __graft_entry__.build())")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7), loaded
    # by file name.  Loaded first, it satisfies the engine's libamdhip64.so.7 dependency; loaded after the
    # engine's /opt/rocm copy, the process holds two runtimes and the second to initialise sees no device.
    # (NEP_HOST_INPUTS=1: host-array descriptors and no PyTorch, the engine on /opt/rocm's runtime — for A/B)
    if not _host_inputs():
        import torch  # noqa: F401
    lib = ctypes.CDLL(p)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    pi32, pi64 = ctypes.POINTER(i32), ctypes.POINTER(i64)
    lib.nep_model_create.argtypes = [ctypes.POINTER(ModelDesc), i32, vp, ctypes.POINTER(vp)]
    lib.nep_model_destroy.argtypes = [vp]
    lib.nep_model_destroy.restype = None
    lib.nep_model_get_info.argtypes = [vp, ctypes.POINTER(ModelInfo)]
    lib.nep_lp_solve_batch.argtypes = [vp, i32, ctypes.POINTER(i32), _dp, _dp, ctypes.POINTER(LpOpts), _dp, _dp,
                                       ctypes.POINTER(i32), ctypes.POINTER(i64)]
    lib.nep_lp_submit.argtypes = [vp, i32, pi32, _dp, _dp, ctypes.POINTER(LpOpts), pi32]
    lib.nep_lp_submit_ex.argtypes = [vp, i32, pi32, _dp, _dp, ctypes.POINTER(LpOpts), pi64, _dp, pi32]
    lib.nep_lp_advance.argtypes = [vp, i32, pi32, pi32, _dp, _dp, pi32, pi64]
    lib.nep_lp_active.argtypes = [vp]
    lib.nep_lp_get_solution.argtypes = [vp, i32, _dp, ctypes.POINTER(ctypes.c_float)]
    lib.nep_lp_get_rows.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i32),
                                    ctypes.POINTER(i32)]
    lib.nep_lp_copy_state.argtypes = [vp, i32, i32]
    lib.nep_lp_copy_states.argtypes = [vp, i32, vp, vp]
    lib.nep_lp_get_flows_solutions.argtypes = [vp, i32, vp, vp, vp]
    lib.nep_lp_copy_routing.argtypes = [vp, i32, vp, i32]
    lib.nep_lp_get_solutions.argtypes = [vp, i32, pi32, _dp]
    lib.nep_round_leaves.argtypes = [i32, i32, _dp, _dp, ctypes.POINTER(ctypes.c_float), _dp, _dp, _dp, i32, pi32, _dp,
                                     _dp, _dp, pi32]
    lib.nep_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    lib.nep_reset_stats.argtypes = [vp]
    lib.nep_reset_stats.restype = None
    lib.nep_lp_get_diag.argtypes = [vp, i32, _dp]
    lib.nep_debug_sparse_rows.argtypes = [vp, i32, vp, vp]
    lib.nep_debug_build.argtypes = [ctypes.POINTER(ModelDesc), _dp, _dp, _dp, _dp, ctypes.POINTER(i32)]
    lib.nep_debug_state.argtypes = [vp, i32, _dp, _dp, ctypes.POINTER(ctypes.c_float), _dp, _dp]
    lib.nep_debug_presolve.argtypes = [ctypes.POINTER(ModelDesc), i32, _dp, _dp, pi32, pi32, _dp, _dp]
    lib.nep_lp_set_params.argtypes = [vp, ctypes.c_double, ctypes.c_double]
    lib.nep_lp_set_reference_weight.argtypes = [vp, ctypes.c_double]
    lib.nep_bnb_create.argtypes = [vp, vp, ctypes.POINTER(BnbParams), _dp, _dp]
    lib.nep_bnb_create.restype = vp
    lib.nep_bnb_destroy.argtypes = [vp]
    lib.nep_bnb_destroy.restype = None
    lib.nep_bnb_add_leaf.argtypes = [vp, i32, pi32, _dp, ctypes.c_double, i32]
    lib.nep_bnb_set_incumbent.argtypes = [vp, ctypes.c_double]
    lib.nep_bnb_event_data.argtypes = [vp, _dp, ctypes.POINTER(ctypes.c_float)]
    lib.nep_bnb_run.argtypes = [vp, pi32]
    lib.nep_bnb_get_stats.argtypes = [vp, ctypes.POINTER(BnbStats)]
    lib.nep_bnb_get_lp_iters.argtypes = [vp, pi64]
    lib.nep_bnb_incumbent.argtypes = [vp, _dp, pi32, pi32, _dp]
    lib.nep_bnb_set_step2.argtypes = [vp, i32, ctypes.c_double, _dp, i32]
    lib.nep_bnb_incumbent_event.argtypes = [vp, pi32, pi32, _dp, _dp]
    lib.nep_bnb_debug_ibound.argtypes = [ctypes.POINTER(BnbParams), i32, ctypes.c_double, _dp, i32, pi32, _dp, _dp]
    lib.nep_bnb_create_engines.argtypes = [ctypes.POINTER(BnbEngine), ctypes.POINTER(BnbEngine),
                                           ctypes.POINTER(BnbParams), _dp, _dp]
    lib.nep_bnb_create_engines.restype = vp
    lib.nep_bnb_sync_get.argtypes = [vp, _dp]
    lib.nep_bnb_sync_set.argtypes = [vp, ctypes.c_double, i32, i64]
    lib.nep_bnb_export_nodes.argtypes = [vp, i32, i32, pi32, _dp, pi32, _dp]
    lib.nep_bnb_import_nodes.argtypes = [vp, i32, pi32, _dp, pi32, _dp]
    lib.nep_lp_get_flows.argtypes = [vp, i32, pi32, ctypes.POINTER(ctypes.c_float)]
    lib.nep_lp_get_flows_split.argtypes = [vp, i32, pi32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.nep_lp_routing_entries.argtypes = [vp, i32, ctypes.c_double, i32, i64, pi64, pi32, pi32, _dp]
    lib.nep_lp_allocation_entries.argtypes = [vp, i32, ctypes.c_double, i64, pi64, pi32, pi32]
    lib.nep_lp_score_check.argtypes = [vp, i32, _dp]
    lib.nep_round_leaf.argtypes = [i32, i32, _dp, _dp, ctypes.POINTER(ctypes.c_float), _dp, _dp, _dp, i32,
                                   ctypes.c_double, _dp, _dp]
    lib.nep_last_error.restype = ctypes.c_char_p
    lib.nep_api_version.restype = ctypes.c_int
    # array arguments travel as plain addresses (_ptr: the array's data pointer as an int): ctypes' typed
    # pointer casts cost ~2 us each, ~10 % of the B&B's host time at 64x32 (tools/probes/bnb_profile.py)
    scalar_ptrs = tuple(ctypes.POINTER(t) for t in (ctypes.c_double, ctypes.c_float, ctypes.c_int32, ctypes.c_int64))
    for name in EXPORTS:
        fn = getattr(lib, name)
        if fn.argtypes:
            fn.argtypes = [ctypes.c_void_p if t in scalar_ptrs else t for t in fn.argtypes]
    if lib.nep_api_version() != API_VERSION:
        raise EngineUnavailable(f"{p}: API version {lib.nep_api_version()} != {API_VERSION} (rebuild the engine)")
    if path is None:
        _lib = lib
    return lib


def round_leaf(c_fix, n_fix, flow, zc, fn_mem, node_mem, by_flow, flow_threshold):
    """The B&B rounding heuristic (nep_round_leaf, host code of the engine library): c_fix [F, N] / n_fix [N]
    (None: no n) with -1 free and 0 / 1 fixed, flow [F, N], zc [F, N] (None: 0).  Returns (c [F*N], n [N] or
    None) or None when the node has no leaf."""
    lib = load_library()
    c_fix = np.ascontiguousarray(c_fix, np.float64)
    F, N = c_fix.shape
    nf = None if n_fix is None else np.ascontiguousarray(n_fix, np.float64)
    fl = np.ascontiguousarray(flow, np.float32)
    zcv = None if zc is None else np.ascontiguousarray(zc, np.float64)
    fm = np.ascontiguousarray(fn_mem, np.float64)
    nm = np.ascontiguousarray(node_mem, np.float64)
    c_out = np.zeros(F * N)
    n_out = None if nf is None else np.zeros(N)
    rc = lib.nep_round_leaf(F, N, _ptr(c_fix), _ptr(nf), _ptr(fl, ctypes.c_float), _ptr(zcv), _ptr(fm), _ptr(nm),
                            1 if by_flow else 0, float(flow_threshold), _ptr(c_out), _ptr(n_out))
    if rc < 0:
        raise EngineUnavailable(f"nep_round_leaf failed ({rc})")
    return (c_out, n_out) if rc == 1 else None


def round_leaves(c_fix, n_fix, flow, zc, fn_mem, node_mem, modes):
    """round_leaf for several (by_flow, flow_threshold) modes of one node in one call (nep_round_leaves):
    [(c, n or None) or None per mode]."""
    lib = load_library()
    c_fix = np.ascontiguousarray(c_fix, np.float64)
    F, N = c_fix.shape
    k = len(modes)
    nf = None if n_fix is None else np.ascontiguousarray(n_fix, np.float64)
    fl = np.ascontiguousarray(flow, np.float32)
    zcv = None if zc is None else np.ascontiguousarray(zc, np.float64)
    bf = np.array([1 if m[0] else 0 for m in modes], np.int32)
    th = np.array([float(m[1]) for m in modes], np.float64)
    # (every converted array is bound to a local first: _ptr passes a raw address, which does not keep a
    # temporary copy alive through the call)
    fm = np.ascontiguousarray(fn_mem, np.float64)
    nm = np.ascontiguousarray(node_mem, np.float64)
    c_out = np.zeros((k, F * N))
    n_out = None if nf is None else np.zeros((k, N))
    found = np.zeros(k, np.int32)
    rc = lib.nep_round_leaves(F, N, _ptr(c_fix), _ptr(nf), _ptr(fl), _ptr(zcv), _ptr(fm), _ptr(nm), k, _ptr(bf),
                              _ptr(th), _ptr(c_out), _ptr(n_out), _ptr(found))
    if rc < 0:
        raise EngineUnavailable(f"nep_round_leaves failed ({rc})")
    return [((c_out[q], None if n_out is None else n_out[q]) if found[q] else None) for q in range(k)]


def _ptr(a, ctype=ctypes.c_double):
    """The data address of a C-contiguous numpy array (the library's array arguments are void*), or None.
    (ctype documents the element type the C side reads.)"""
    return None if a is None else a.ctypes.data


def _check(lib, rc, what):
    if rc != 0:
        raise EngineUnavailable(f"{what} failed ({rc}): {lib.nep_last_error().decode()}")


def _arrays(data, N, F):
    f64 = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return dict(
        delay=f64(data.node_delay_matrix).reshape(N, N),
        workload=f64(data.workload_matrix).reshape(F, N),
        cpr=f64(data.core_per_req_matrix).reshape(F, N),
        fmem=f64(data.function_memory_matrix).reshape(F),
        nmem=f64(data.node_memory_matrix).reshape(N),
        ncores=f64(data.node_cores_matrix).reshape(N),
        ncost=f64(data.node_costs).reshape(N),
        maxd=f64(data.max_delay_matrix).reshape(F),
        old=f64(data.old_allocations_matrix).reshape(F, N),
    )


def _desc(k, N, F, variant, step, alpha, soften, max_score, prev_delay, budget, relaxation=RELAX_REFERENCE):
    """The model descriptor over host numpy arrays, or (API 9, device_inputs = 1) over the device memory of
    PyTorch-ROCm tensors (instance_tensors)."""
    dev = not isinstance(k["delay"], np.ndarray)

    def dp(a):   # (structure fields keep their typed pointers)
        return ctypes.cast(ctypes.c_void_p(a.data_ptr()), _dp) if dev else a.ctypes.data_as(_dp)
    return ModelDesc(N, F, variant, step, float(alpha), float(soften), float(max_score), float(prev_delay), 1e6,
                     1e-6, dp(k["delay"]), dp(k["workload"]), dp(k["cpr"]), dp(k["fmem"]), dp(k["nmem"]),
                     dp(k["ncores"]), dp(k["ncost"]), float(budget), dp(k["maxd"]), dp(k["old"]),
                     int(relaxation), 1 if dev else 0)


def instance_tensors(data, device=None):
    """The instance of a Data (core/utils/data.py; input_to_data.py:88-111) as contiguous float64 PyTorch-ROCm
    tensors on the GPU — the constraint data the engine's models are built from (nep_model_desc.device_inputs):
    D [N, N], W [F, N], core_per_req [F, N], function memory [F], node memory / cores / costs [N], max delay
    [F], old allocations [F, N].  Requires a GPU (the product path has no CPU fallback)."""
    import torch
    if not torch.cuda.is_available():
        raise EngineUnavailable("no GPU visible: the engine's instance tensors live on the device")
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    host = _arrays(data, len(data.nodes), len(data.functions))
    out = {k: torch.from_numpy(v).to(dev).contiguous() for k, v in host.items()}
    torch.cuda.synchronize(dev)   # (the library reads them on its own streams)
    return out


def debug_build(data, variant, step=STEP1, alpha=0.5, soften_step1_sol=1.3, max_score=0.0, prev_network_delay=0.0,
                relaxation=RELAX_REFERENCE):
    """Host-only model build (no GPU needed): returns eta, rho, gam, rownorm, dims."""
    lib = load_library()
    N, F = len(data.nodes), len(data.functions)
    v = VARIANTS[variant] if isinstance(variant, str) else int(variant)
    k = _arrays(data, N, F)
    d = _desc(k, N, F, v, int(step), alpha, soften_step1_sol, max_score, prev_network_delay, data.node_budget,
              relaxation)
    dims = np.zeros(4, np.int32)
    eta = np.zeros(1)
    _check(lib, lib.nep_debug_build(ctypes.byref(d), _ptr(eta), None, None, None, _ptr(dims, ctypes.c_int32)),
           "nep_debug_build")
    R, T, n_int, n_dual = dims.tolist()
    rho, gam, rn = np.zeros(n_dual), np.zeros(n_int), np.zeros(n_dual)
    _check(lib, lib.nep_debug_build(ctypes.byref(d), _ptr(eta), _ptr(rho), _ptr(gam), _ptr(rn), None),
           "nep_debug_build")
    return {"eta": float(eta[0]), "rho": rho, "gam": gam, "rownorm": rn, "R": R, "T": T, "n_int": n_int,
            "n_dual": n_dual}


def debug_presolve(data, variant, lb, ub, step=STEP1, alpha=0.5, soften_step1_sol=1.3, max_score=0.0,
                   prev_network_delay=0.0):
    """Host-only node presolve of [n, n_int] node bounds, from scratch and as the sparse change of
    the base box nep_lp_submit uses: returns (ok_full, ok_node, box_full, box_node)."""
    lib = load_library()
    N, F = len(data.nodes), len(data.functions)
    v = VARIANTS[variant] if isinstance(variant, str) else int(variant)
    k = _arrays(data, N, F)
    d = _desc(k, N, F, v, int(step), alpha, soften_step1_sol, max_score, prev_network_delay, data.node_budget)
    lb = np.ascontiguousarray(lb, np.float64)
    ub = np.ascontiguousarray(ub, np.float64)
    n, ni = lb.shape
    okf = np.zeros(n, np.int32)
    okn = np.zeros(n, np.int32)
    bf = np.zeros((n, 2, ni))
    bn = np.zeros((n, 2, ni))
    _check(lib, lib.nep_debug_presolve(ctypes.byref(d), n, _ptr(lb), _ptr(ub), _ptr(okf, ctypes.c_int32),
                                       _ptr(okn, ctypes.c_int32), _ptr(bf), _ptr(bn)), "nep_debug_presolve")
    return okf.astype(bool), okn.astype(bool), bf, bn


class LPModel:
    """One structured LP family (a reference step model) with `max_batch` device slots."""

    def __init__(self, data, variant, step=STEP1, alpha=0.5, soften_step1_sol=1.3, max_score=0.0,
                 prev_network_delay=0.0, max_batch=1, relaxation=RELAX_REFERENCE):
        self._lib = load_library()
        self.N = len(data.nodes)
        self.F = len(data.functions)
        self.variant = VARIANTS[variant] if isinstance(variant, str) else int(variant)
        self.step = int(step)
        self._keep = _arrays(data, self.N, self.F)
        # the instance as PyTorch-ROCm tensors: the library builds the model from their device memory
        # (nep_model_desc.device_inputs, API 9)
        self.tensors = None if _host_inputs() else instance_tensors(data)
        self.relaxation = int(relaxation)
        d = _desc(self._keep if self.tensors is None else self.tensors, self.N, self.F, self.variant, self.step, alpha, soften_step1_sol, max_score,
                  prev_network_delay, data.node_budget, self.relaxation)
        h = ctypes.c_void_p()
        _check(self._lib, self._lib.nep_model_create(ctypes.byref(d), int(max_batch), None, ctypes.byref(h)),
               "nep_model_create")
        self._h = h
        info = ModelInfo()
        _check(self._lib, self._lib.nep_model_get_info(self._h, ctypes.byref(info)), "nep_model_get_info")
        self.info = info
        self.n_int = info.n_int
        self.max_batch = info.max_batch

    def close(self):
        if getattr(self, "_h", None):
            self._lib.nep_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _bounds(self, B, lb, ub):
        lbp = None if lb is None else np.ascontiguousarray(np.asarray(lb, np.float64).reshape(B, self.n_int))
        ubp = None if ub is None else np.ascontiguousarray(np.asarray(ub, np.float64).reshape(B, self.n_int))
        return lbp, ubp

    def solve(self, slots, lb=None, ub=None, tol=1e-7, cutoff=math.inf, max_iters=200000, check_every=64,
              warm_start=False, warm_omega_floor=0.0, gap_tol=0.0, warm_omega_cap=0.0, polish_after=0.0,
              bound_res=0.0):
        """Solve len(slots) node LPs.  lb/ub: [B, n_int] bounds on the integer vector (None = root).
        Returns dict of numpy arrays: obj (certified LP value = Lagrangian bound), primal_obj, status, iters."""
        slots = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).reshape(-1))
        B = len(slots)
        lbp, ubp = self._bounds(B, lb, ub)
        obj = np.zeros(B)
        pobj = np.zeros(B)
        status = np.zeros(B, np.int32)
        iters = np.zeros(B, np.int64)
        opts = LpOpts(float(tol), float(cutoff), int(max_iters), int(check_every), 1 if warm_start else 0,
                      float(warm_omega_floor), float(gap_tol), float(warm_omega_cap), float(polish_after),
                      float(bound_res))
        _check(self._lib, self._lib.nep_lp_solve_batch(
            self._h, B, _ptr(slots, ctypes.c_int32), _ptr(lbp), _ptr(ubp), ctypes.byref(opts), _ptr(obj), _ptr(pobj),
            _ptr(status, ctypes.c_int32), _ptr(iters, ctypes.c_int64)), "nep_lp_solve_batch")
        return {"obj": obj, "primal_obj": pobj, "status": status, "iters": iters}

    # streaming form (nep_lp_submit / nep_lp_advance): a B&B keeps every slot busy
    def submit(self, slots, lb=None, ub=None, tol=1e-7, cutoff=math.inf, max_iters=200000, check_every=64,
               warm_start=False, warm_omega_floor=0.0, gap_tol=0.0, warm_omega_cap=0.0, polish_after=0.0,
              bound_res=0.0):
        """Start node LPs in free slots; returns their presolve status (LP_INFEASIBLE: proven
        infeasible, not started; LP_ITERATION_LIMIT: iterating).  max_iters / bound_res may be per-LP
        arrays (length len(slots)): then one nep_lp_submit_ex call (API 12) carries them."""
        slots = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).reshape(-1))
        B = len(slots)
        lbp, ubp = self._bounds(B, lb, ub)
        status = np.zeros(B, np.int32)
        per = np.ndim(max_iters) > 0 or np.ndim(bound_res) > 0
        mi = np.ascontiguousarray(np.broadcast_to(np.asarray(max_iters, np.int64), (B,))) if per else None
        br = np.ascontiguousarray(np.broadcast_to(np.asarray(bound_res, np.float64), (B,))) if per else None
        opts = LpOpts(float(tol), float(cutoff), int(mi.max()) if per and B else int(np.max(max_iters)),
                      int(check_every), 1 if warm_start else 0, float(warm_omega_floor), float(gap_tol),
                      float(warm_omega_cap), float(polish_after), 0.0 if per else float(bound_res))
        if per:
            _check(self._lib, self._lib.nep_lp_submit_ex(self._h, B, _ptr(slots, ctypes.c_int32), _ptr(lbp), _ptr(ubp),
                                                         ctypes.byref(opts), _ptr(mi, ctypes.c_int64), _ptr(br),
                                                         _ptr(status, ctypes.c_int32)), "nep_lp_submit_ex")
            return status
        _check(self._lib, self._lib.nep_lp_submit(self._h, B, _ptr(slots, ctypes.c_int32), _ptr(lbp), _ptr(ubp),
                                                  ctypes.byref(opts), _ptr(status, ctypes.c_int32)),
               "nep_lp_submit")
        return status

    def advance(self, min_done=1):
        """Iterate until at least `min_done` LPs finished (0: one block of check_every iterations).
        Returns the finished slots and their results."""
        mb = self.max_batch
        n = ctypes.c_int32(0)
        slots = np.zeros(mb, np.int32)
        obj = np.zeros(mb)
        pobj = np.zeros(mb)
        status = np.zeros(mb, np.int32)
        iters = np.zeros(mb, np.int64)
        _check(self._lib, self._lib.nep_lp_advance(self._h, int(min_done), ctypes.byref(n),
                                                   _ptr(slots, ctypes.c_int32), _ptr(obj), _ptr(pobj),
                                                   _ptr(status, ctypes.c_int32), _ptr(iters, ctypes.c_int64)),
               "nep_lp_advance")
        k = n.value
        return {"slots": slots[:k], "obj": obj[:k], "primal_obj": pobj[:k], "status": status[:k],
                "iters": iters[:k]}

    def active(self):
        """Number of slots iterating (submitted and not yet finished)."""
        return int(self._lib.nep_lp_active(self._h))

    def solution(self, slot, dense_x=True):
        z = np.zeros(self.n_int)
        x = np.zeros((self.N, self.F, self.N), np.float32) if dense_x else None
        _check(self._lib, self._lib.nep_lp_get_solution(self._h, int(slot), _ptr(z),
                                                        _ptr(x, ctypes.c_float) if dense_x else None),
               "nep_lp_get_solution")
        return z, x

    def solutions(self, slots):
        """z_int of several finished slots, [len(slots), n_int], in one device round trip (nep_lp_get_solutions)."""
        slots = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).reshape(-1))
        out = np.zeros((len(slots), self.n_int))
        _check(self._lib, self._lib.nep_lp_get_solutions(self._h, len(slots), _ptr(slots, ctypes.c_int32), _ptr(out)),
               "nep_lp_get_solutions")
        return out

    def rows(self, slot):
        R = self.info.n_rows
        xb = np.zeros((R, self.N), np.float32)
        rf = np.zeros(R, np.int32)
        rs = np.zeros(R, np.int32)
        _check(self._lib, self._lib.nep_lp_get_rows(self._h, int(slot), _ptr(xb, ctypes.c_float),
                                                    _ptr(rf, ctypes.c_int32), _ptr(rs, ctypes.c_int32)),
               "nep_lp_get_rows")
        return xb, rf, rs

    def row_map(self):
        """(row_f, row_src) of the aggregated routing rows (src = -1: the pooled zero-workload sources)."""
        if getattr(self, "_rowmap", None) is None:
            R = self.info.n_rows
            rf = np.zeros(R, np.int32)
            rs = np.zeros(R, np.int32)
            _check(self._lib, self._lib.nep_lp_get_rows(self._h, 0, None, _ptr(rf, ctypes.c_int32),
                                                        _ptr(rs, ctypes.c_int32)), "nep_lp_get_rows")
            self._rowmap = (rf, rs)
        return self._rowmap

    def routing_from_entries(self, row, dst, val):
        from .routing import SparseRouting
        rf, rs = self.row_map()
        return SparseRouting(self.N, self.F, rf, rs, self._keep["workload"], row, dst, val)

    def routing(self, slot):
        """The slot's routing x[i][f][j] as a SparseRouting: every nonzero of the aggregated rows, compacted
        on the device (nep_lp_routing_entries, threshold 0, unrounded) — the dense N*F*N matrix never
        crosses PCIe."""
        row, dst, val = self.routing_entries(slot, threshold=0.0, round3=False)
        return self.routing_from_entries(row, dst, val)

    def set_params(self, tol=1e-7, cutoff=math.inf):
        """tol / cutoff of every LP in flight (nep_lp_set_params): a B&B lowers the cutoff to each new
        incumbent without resubmitting."""
        _check(self._lib, self._lib.nep_lp_set_params(self._h, float(tol), float(cutoff)), "nep_lp_set_params")

    def flows_solutions(self, slots):
        """(flows(slots), solutions(slots)) in one device round trip (nep_lp_get_flows_solutions)."""
        slots = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).reshape(-1))
        fl = np.zeros((len(slots), self.F, self.N), np.float32)
        z = np.zeros((len(slots), self.n_int))
        _check(self._lib, self._lib.nep_lp_get_flows_solutions(self._h, len(slots), _ptr(slots, ctypes.c_int32),
                                                               _ptr(fl, ctypes.c_float), _ptr(z)),
               "nep_lp_get_flows_solutions")
        return fl, z

    def flows(self, slots, split=False):
        """flow[b, f, j] = sum_i x[i, f, j] of finished slots, reduced on the device (nep_lp_get_flows);
        split=True: (flow, workload-source part of it) (nep_lp_get_flows_split)."""
        slots = np.ascontiguousarray(np.asarray(slots, dtype=np.int32).reshape(-1))
        out = np.zeros((len(slots), self.F, self.N), np.float32)
        if split:
            wout = np.zeros_like(out)
            _check(self._lib, self._lib.nep_lp_get_flows_split(
                self._h, len(slots), _ptr(slots, ctypes.c_int32), _ptr(out, ctypes.c_float),
                _ptr(wout, ctypes.c_float)), "nep_lp_get_flows_split")
            return out, wout
        _check(self._lib, self._lib.nep_lp_get_flows(self._h, len(slots), _ptr(slots, ctypes.c_int32),
                                                     _ptr(out, ctypes.c_float)), "nep_lp_get_flows")
        return out

    def routing_entries(self, slot, threshold=0.001, round3=True):
        """Compacted routing entries of the aggregated rows, x > threshold, on the device
        (nep_lp_routing_entries; neptune/utils/output.py:23-31): (row, dst, value) arrays."""
        n = ctypes.c_int64(0)
        _check(self._lib, self._lib.nep_lp_routing_entries(self._h, int(slot), float(threshold), int(round3), 0,
                                                           ctypes.byref(n), None, None, None), "nep_lp_routing_entries")
        k = n.value
        row = np.zeros(k, np.int32)
        dst = np.zeros(k, np.int32)
        val = np.zeros(k)
        if k:
            _check(self._lib, self._lib.nep_lp_routing_entries(
                self._h, int(slot), float(threshold), int(round3), k, ctypes.byref(n), _ptr(row, ctypes.c_int32),
                _ptr(dst, ctypes.c_int32), _ptr(val)), "nep_lp_routing_entries")
        return row, dst, val

    def allocation_entries(self, slot, threshold=0.001):
        """(f, j) pairs with c[f, j] > threshold, compacted on the device (output.py:33-39)."""
        n = ctypes.c_int64(0)
        _check(self._lib, self._lib.nep_lp_allocation_entries(self._h, int(slot), float(threshold), 0,
                                                              ctypes.byref(n), None, None),
               "nep_lp_allocation_entries")
        k = n.value
        fn = np.zeros(k, np.int32)
        dst = np.zeros(k, np.int32)
        if k:
            _check(self._lib, self._lib.nep_lp_allocation_entries(
                self._h, int(slot), float(threshold), k, ctypes.byref(n), _ptr(fn, ctypes.c_int32),
                _ptr(dst, ctypes.c_int32)), "nep_lp_allocation_entries")
        return fn, dst

    def score_check(self, slot):
        """The reference's scorers and feasibility checkers on a slot's solution, on the device
        (nep_lp_score_check; efttc/utils/objectives.py, efttc/utils/constraints_step1.py)."""
        out = np.zeros(len(SCORE_FIELDS))
        _check(self._lib, self._lib.nep_lp_score_check(self._h, int(slot), _ptr(out)), "nep_lp_score_check")
        return dict(zip(SCORE_FIELDS, out.tolist()))

    DIAG = ("pobj", "lagr", "best_lagr", "pres", "gap", "omega", "tau", "sigma", "eta", "k", "k_since_restart",
            "status", "active", "restart_fpr", "last_fpr", "sigma_max")

    def sparse_rows(self, slot):
        """Per routing row of a slot: the nonzeros its Halpern anchor is held with (kAnchorDense = 17: the row is
        dense) and (facility relaxation) the nonzeros of its x <= c duals."""
        R = self.info.n_rows
        a = np.zeros(R, np.int32)
        lam = np.zeros(R, np.float32) if self.relaxation == RELAX_FACILITY else None
        _check(self._lib, self._lib.nep_debug_sparse_rows(self._h, int(slot), _ptr(a), _ptr(lam)),
               "nep_debug_sparse_rows")
        return a, lam

    def diag(self, slot):
        out = np.zeros(16)
        _check(self._lib, self._lib.nep_lp_get_diag(self._h, int(slot), _ptr(out)), "nep_lp_get_diag")
        return dict(zip(self.DIAG, out.tolist()))

    def debug_state(self, slot, n_dual):
        """Device state of a slot (nep_debug_state): duals y, row activities kz, node bounds lb / ub."""
        y, kz = np.zeros(n_dual), np.zeros(n_dual)
        lb, ub = np.zeros(self.n_int), np.zeros(self.n_int)
        _check(self._lib, self._lib.nep_debug_state(self._h, int(slot), _ptr(y), _ptr(kz), None, _ptr(lb), _ptr(ub)),
               "nep_debug_state")
        return {"y": y, "kz": kz, "lb": lb, "ub": ub}

    def set_reference_weight(self, omega_ref):
        """Warm starts take their primal weight in [floor, cap] x omega_ref (nep_lp_set_reference_weight, API 10);
        0: relative to the parent's final weight."""
        _check(self._lib, self._lib.nep_lp_set_reference_weight(self._h, float(omega_ref)),
               "nep_lp_set_reference_weight")

    def copy_state(self, src, dst):
        _check(self._lib, self._lib.nep_lp_copy_state(self._h, int(src), int(dst)), "nep_lp_copy_state")

    def copy_states(self, src, dst):
        """copy_state(src[k], dst[k]) for every k, in order, in as few launches as the pairs allow
        (nep_lp_copy_states)."""
        src = np.ascontiguousarray(np.asarray(src, np.int32).reshape(-1))
        dst = np.ascontiguousarray(np.asarray(dst, np.int32).reshape(-1))
        if src.size != dst.size:
            raise ValueError("copy_states: src and dst differ in length")
        _check(self._lib, self._lib.nep_lp_copy_states(self._h, int(src.size), _ptr(src, ctypes.c_int32),
                                                       _ptr(dst, ctypes.c_int32)), "nep_lp_copy_states")

    def copy_routing_from(self, other, src, dst):
        """x and thresholds of slot `src` of model `other` (same instance and rows, e.g. the facility
        relaxation's) into this model's slot `dst` (nep_lp_copy_routing)."""
        _check(self._lib, self._lib.nep_lp_copy_routing(self._h, int(dst), other._h, int(src)), "nep_lp_copy_routing")

    def stats(self):
        s = Stats()
        _check(self._lib, self._lib.nep_get_stats(self._h, ctypes.byref(s)), "nep_get_stats")
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    def reset_stats(self):
        self._lib.nep_reset_stats(self._h)

    # integer-vector layout helpers (include/neptune_lp.h)
    def layout(self):
        FN, N = self.F * self.N, self.N
        has_n = self.variant != MIN_DELAY
        if self.step == STEP1:
            return {"c": (0, FN), "n": (FN, FN + N) if has_n else None}
        out = {"c": (0, FN), "moved_from": (FN, 2 * FN), "moved_to": (2 * FN, 3 * FN),
               "allocated": (3 * FN, 3 * FN + 1), "deallocated": (3 * FN + 1, 3 * FN + 2)}
        out["n"] = (3 * FN + 2, 3 * FN + 2 + N) if has_n else None
        return out
