#!/usr/bin/env python3
"""bench.py — LP-relaxations/sec (+ certified objective gap) on the synthetic 512-node x
256-function NEPTUNE instance (BASELINE.json `metric`; generator of SURVEY.md §8(d)).

Workload (`value`).  The node LPs the product's own branch-and-bound submitted on this instance
(step-1 NeptuneMinDelayAndUtilization, reference `core/solvers/neptune/neptune_step1.py:67-77`, rows
`neptune/utils/constraints_step1.py`, objective `neptune/utils/objectives.py:30-52`), recorded by
tools/record_bnb_trace.py into tests/golden/bnb_trace_512x256_s0.json.gz (s1: `--seed 1`) and REPLAYED in
submission order, except that a box waits while its parent's LP still iterates (the B&B creates a node only once
its parent finished; later ready boxes go first; `--in-order` disables this): each recorded box (a branching node's fixings; a leaf's open c and n, every other c and n fixed to
0) is solved as an LP relaxation of the REFERENCE model — the LP SCIP solves at that node
(core/solvers/solver.py:35-40).  `--batch` node LPs are in flight per GPU (nep_lp_submit /
nep_lp_advance): a slot whose LP finishes takes the next box at once.  A node starts from its parent's
final PDHG state when a slot still holds it (slots are refilled oldest-finished first; finished parents
with open children are parked, `--park` slots), else from the root's, with the PDHG primal weight banded around
8 x the model's cold-start weight (`--omega-ref`, nep_lp_set_reference_weight).  The timed region
streams the WHOLE recorded trace once (1026 node LPs at 512x256, seed 0) and drains it, whatever --steps says:
one *step* is 1/K of the trace (ms_per_step = wall / K), so `value` does not depend on --steps / --warmup (the
warmup streams the first W x --batch boxes on a stream of its own, untimed).  A node counts only if the engine
certifies it: repaired primal objective - Lagrangian bound <= tol*max(1,|bound|) and every row residual <= tol
(DESIGN.md §4); nodes that stop at `--max-iters` keep a valid bound and are reported, not counted.  The root LP
is solved before the timed region (its seconds are `lp.root_seconds`); the instance lives on the device before
the timer starts; node bounds are uploaded inside it, as the B&B host does per node.  Secondary figures in the
same JSON: `product_node_lp_per_s` (the product search's own node-LP rates), `native_replay` (the trace's first
boxes on the models the product ran them on), `children_stream` (root children with `--fix` random c-fixings,
the round-1..3 workload), `bnb` (the product search itself) and `alibaba_flows` (the reference's three Alibaba
requests end to end beside its published processing_time).

Multi-GPU.  `--gpus N` > 1 without a launcher environment starts N rank processes itself
(torch.distributed.run, one rank per GPU, 127.0.0.1 rendezvous) before anything touches the GPU; under a
launcher the world it reports must equal --gpus.  Rank r replays the recorded B&B of instance seed --seed + r
(one placement request per GPU: weak scaling; `rank_seed`); the only exchange is the B&B bound all-reduce(MIN)
of 8 bytes per timed stream.  value = certified LPs of all ranks / max-over-ranks wall time.  The sharded search
of ONE instance (subtrees per rank, one packed all-reduce per loop over RCCL) is the `bnb` section.

Roofline.  The dominant kernel is `x_pass` (csrc/nep_kernels.hip).  Its algorithmic bytes per LP
iteration are SURVEY.md §8(d)'s B_iter = 4 (2P + 2FN + 2N + 2m) (x, c, n and the duals, each read and
written, fp32 units; P = R*N routing entries after exact zero-workload aggregation, m = the dualised rows;
nep_model_info.bytes_per_iter: 58.7 MB at 512x256).  `achieved` = B_iter x the LPs one sampled launch
carries / that launch's HIP-event duration on the engine's own stream, averaged over one steady-state
launch per block (nep_get_stats).  `traffic` is read from profiles/traffic.json (separate rocprofv3 --pmc
passes, tools/traffic.py) when it was measured on this exact workload (else null), per
LP-iteration and scaled to the LPs of the average sampled launch.

CPU baseline.  The oracle (HiGHS on the reference's formulation restated as one CSR, oracle/) timed on
rank 0's host, bounded by `--cpu-budget` seconds (see `cpu_baseline`).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "neptune-mip_amd")
for _p in (PKG, REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--nodes", type=int, default=512)
    ap.add_argument("--functions", type=int, default=256)
    ap.add_argument("--batch", type=int, default=32, help="node LPs in flight per GPU (= node LPs per step)")
    ap.add_argument("--fix", type=int, default=2, help="c[f,j] fixings per node LP")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--max-iters", type=int, default=8192,
                    help="per node LP of the timed streams (a B&B node-LP iteration limit; nodes that reach it keep "
                         "a valid Lagrangian bound but are not counted as LP relaxations).  Replay, check every 48: "
                         "2048 / 4096 / 8192 / 12288 / 16384 / 32768 -> 5.96 / 7.07 / 8.23 / 8.03 / 7.53 / 6.34 "
                         "certified LP/s (DESIGN.md §6)")
    ap.add_argument("--bnb-max-iters", type=int, default=4096,
                    help="the bnb section's node-LP limit (leaves; branching nodes a quarter of it), as the replay "
                         "trace was recorded")
    ap.add_argument("--warm-omega-floor", type=float, default=0.0,
                    help="warm-start primal-weight floor x the parent's (0: engine default)")
    ap.add_argument("--omega-ref", type=float, default=8.0,
                    help="warm starts take their primal weight in [floor, cap] x (this x the model's cold-start weight "
                         "omega0) (nep_lp_set_reference_weight; 0: relative to the parent's final weight)")
    ap.add_argument("--leaf-omega", default="",
                    help="replay: warm-start weight band of leaf boxes (every c and n fixed) as 'floor:cap' multiples "
                         "of the reference weight (default: the engine's 2,4 for every box)")
    ap.add_argument("--polish-after", type=float, default=0.0,
                    help="replay: warm-started node LPs start primal-feasibility polishing after this many iterations "
                         "(0: the engine's default, 256; -1: never)")
    ap.add_argument("--root-max-iters", type=int, default=400000)
    ap.add_argument("--check-every", type=int, default=48,
                    help="PDHG iterations per certificate check of the timed streams (replay: 12 / 24 / 48 -> 5.70 / "
                         "6.37 / 7.06 certified LP/s, DESIGN.md §6); the bnb section keeps the product's default")
    ap.add_argument("--root-check-every", type=int, default=64)
    ap.add_argument("--root-polish-after", type=int, default=0,
                    help="primal feasibility polishing of the (cold) root after this many iterations (0: the engine's "
                         "default for cold LPs, none; DESIGN.md §4 'Polishing')")
    ap.add_argument("--root-gap-tol", type=float, default=0.0,
                    help="after the root certifies at --tol, continue it (warm, same slot) until its objective gap "
                         "is below this: the children warm-start from a well-converged root (0 = off)")
    ap.add_argument("--cold", action="store_true", help="cold-start every node LP")
    ap.add_argument("--leaf-start", default="parent", choices=("parent", "root", "cold"),
                    help="(A/B) where a replayed rounding leaf starts: its branching node's state (default), the "
                         "root's, or cold")
    ap.add_argument("--stream", default="auto", choices=("auto", "replay", "children"),
                    help="the timed node-LP stream: the product B&B's recorded nodes (replay, tests/golden/"
                         "bnb_trace_<N>x<F>_s<seed>.json.gz) or root children with --fix random fixings; auto: "
                         "replay when the trace exists")
    ap.add_argument("--native-steps", type=int, default=6,
                    help="with the replay stream: steps of the native-model replay timed after it (each recorded "
                         "box on the model the product ran it on; 0 = skip)")
    ap.add_argument("--park", type=int, default=1024,
                    help="replay: slots per model beyond --batch that keep finished nodes' states while their children "
                         "are still to come (warm start from the parent; 0: only free slots keep states).  1024 (76 GB "
                         "of slot state at 512x256): the same warm sources as 256, x_pass launches 6 %% shorter "
                         "(profiles/r05/pad: the working slots' placement, not padding or allocation size)")
    ap.add_argument("--warm-ancestors", action="store_true",
                    help="replay: a node whose parent's state is gone starts from its closest resident ancestor's "
                         "(default: the root's, as the product B&B does)")
    ap.add_argument("--children-steps", type=int, default=24,
                    help="with the replay stream: steps of the children stream timed after it (secondary figure)")
    ap.add_argument("--cpu-budget", type=float, default=150.0,
                    help="seconds for the CPU baseline (0 = skip); the bench-size attempt gets what the fit leaves, "
                         ">= 30 s")
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="CPU baseline worker processes (0: the host's per-GPU share of its cores, cpu_baseline_workers)")
    ap.add_argument("--bnb-seconds", type=float, default=20.0,
                    help="time limit of the product branch-and-bound section (0 = skip)")
    ap.add_argument("--bnb-sizes", default="256x128:20,512x256:60",
                    help="instances of the product B&B section (BASELINE configs 3 and 4), NxF[:seconds] "
                         "comma-separated (seconds: that instance's time limit, default --bnb-seconds)")
    ap.add_argument("--in-order", action="store_true",
                    help="replay: submit the recorded boxes strictly in their recorded order (default: a box waits "
                         "while its parent's LP still iterates, as in the B&B, and later ready boxes go first)")
    ap.add_argument("--dump", default=None, help="write per-node-LP records of the replay (kind, depth, warm source, "
                    "status, iterations, final diagnostics of the uncertified) to this JSON file")
    ap.add_argument("--alibaba-seconds", type=float, default=120.0,
                    help="alibaba_flows section: the reference's three Alibaba 100x25 requests through core.request "
                         "(main.py's route body), each B&B step limited to this many seconds (a safety bound: they end "
                         "OPTIMAL well within it); 0 = skip")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    return ap.parse_args(argv)


def children_workload_name(a):
    return (f"synthetic_{a.nodes}x{a.functions}_step1_MDU_bnb_children_stream_B{a.batch}_fix{a.fix}_"
            f"{'cold' if a.cold else 'warm'}")


def workload_name(a, kind):
    if kind == "replay":
        return f"synthetic_{a.nodes}x{a.functions}_step1_MDU_bnb_node_replay_s{a.seed}_B{a.batch}_reference_lp"
    return children_workload_name(a)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def node_bounds(n_int, F, N, B, k, seed):
    """B children of the root: k distinct c[f,j] fixed to 0/1 each (seeded)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lb = np.full((B, n_int), -np.inf)
    ub = np.full((B, n_int), np.inf)
    for b in range(B):
        idx = rng.choice(F * N, size=k, replace=False)
        val = rng.integers(0, 2, size=k).astype(np.float64)
        lb[b, idx] = val
        ub[b, idx] = val
    return lb, ub


def _dnf_probe(N, F, seed, fix, seconds):
    """One node LP of the bench workload at the bench size on the CPU path itself: the literal reference
    model (oracle/formulation.py, 67 M routing columns / 269 M nonzeros at 512x256) built and handed to
    HiGHS in a child process with a wall budget of `seconds` (HiGHS time_limit + a kill after it).
    Reports its LP time, or "DNF > T" with the stage it reached."""
    import subprocess
    code = ("import sys, time, numpy as np; sys.path[:0]=%r\n"
            "from core.utils.synthetic import synthetic_payload\n"
            "from oracle.inputs import data_to_solver_input\n"
            "from oracle.formulation import build_model\n"
            "from oracle.solve import solve\n"
            "t0=time.perf_counter(); p=synthetic_payload(%d,%d,seed=%d); d=data_to_solver_input(p,with_db=False)\n"
            "m=build_model(d,'MinDelayAndUtilization',step=1,alpha=0.5)\n"
            "print('built', m['A'].shape, m['A'].nnz, time.perf_counter()-t0, flush=True)\n"
            "nx=%d*%d*%d; rng=np.random.default_rng(%d); idx=rng.choice(%d*%d, size=%d, replace=False)\n"
            "lb=m['lb'].copy(); ub=m['ub'].copy(); v=rng.integers(0,2,size=%d).astype(float)\n"
            "lb[nx+idx]=v; ub[nx+idx]=v; t1=time.perf_counter()\n"
            "st,obj,_=solve(m, relax=True, lb=lb, ub=ub, time_limit=max(1.0, %f-(t1-t0)))\n"
            "print('solved', st, obj, time.perf_counter()-t1, flush=True)\n"
            % ([PKG, REPO], N, F, seed, N, N, F, seed, F, N, fix, fix, seconds))
    t0 = time.perf_counter()
    out = {"seconds_budget": seconds, "stage": "model build"}

    def parse(text):
        # (a child killed at the budget still reports the stage it reached: its stdout up to the kill)
        if isinstance(text, bytes):
            text = text.decode(errors="replace")
        for ln in (text or "").splitlines():
            if ln.startswith("built"):
                out["stage"] = "HiGHS LP"
                out["build_s"] = float(ln.split()[-1])
            if ln.startswith("solved"):
                _, st, obj, sec = ln.split()
                out.update(lp_status=int(st), lp_seconds=float(sec))
    try:
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=seconds + 5)
        parse(r.stdout)
    except subprocess.TimeoutExpired as e:
        parse(e.stdout)
    out["finished"] = out.get("lp_status") == 0
    out["wall_s"] = time.perf_counter() - t0
    if "build_s" in out:
        # HiGHS seconds reached: the wall after the build, or its own time_limit status when it returned
        out["highs_s"] = out.get("lp_seconds", out["wall_s"] - out["build_s"])
    if not out["finished"]:
        out["note"] = (f"DNF > {seconds:.0f} s: the {N}x{F} node LP ({N * N * F:,} routing columns) reached "
                       f"'{out['stage']}' and had not finished"
                       + (f" (model built in {out['build_s']:.1f} s, then {out['highs_s']:.1f} s of HiGHS)"
                          if "build_s" in out else ""))
    return out


def cpu_baseline_workers():
    """The CPU baseline's worker processes: this GPU's share of the host's cores — the cores this process may
    run on, divided by the host's GPUs when it is a multi-GPU node (256 cores / 8 MI355X = 32 on the GPU box;
    every core of a host with < 64).  Counted without initialising the GPU."""
    cores = len(os.sched_getaffinity(0))
    total = os.cpu_count() or cores
    gpus = 8 if total >= 64 else 1
    return max(1, min(cores, total // gpus))


def cpu_baseline(N, F, seed, fix, budget, workers):
    """The reference formulation of the same generator, solved by the oracle (HiGHS LP; oracle/).

    1. single-thread node-LP times at growing sizes (same generator, same kind of fixings) -> the
       power-law fit t ~ (N^2 F)^p;
    2. throughput: `workers` node LPs of the largest measured size solved at once, one per worker
       process (oracle/solve.py lp_batch_cpu), i.e. the host's LP/s at that size;
    3. the bench size: a bounded attempt (model build in a child process, killed at the budget's
       share) -> "DNF > T"; the 512x256 LP/s is the measured pool rate scaled by the fitted per-LP
       time ratio."""
    import numpy as np
    from oracle.formulation import build_model
    from oracle.inputs import data_to_solver_input as oracle_input
    from oracle.solve import lp_batch_cpu
    from oracle.solve import solve as oracle_solve
    from core.utils.synthetic import synthetic_payload

    def model_and_bounds(n, f, count, s):
        p = synthetic_payload(n, f, seed=seed)
        d = oracle_input(p, workload_coeff=1, with_db=False)
        m = build_model(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"])
        nx = n * n * f
        lb, ub = node_bounds(f * n + n, f, n, count, fix, seed=s)
        out = []
        for b in range(count):
            rl, ru = m["lb"].copy(), m["ub"].copy()
            fin = np.isfinite(lb[b])
            rl[nx:][fin] = lb[b][fin]
            ru[nx:][fin] = ub[b][fin]
            out.append((rl, ru))
        return m, out

    t_start = time.perf_counter()
    pts = []
    for n in (16, 24, 32, 48, 64, 96, 128, 192, 256):   # (up to BASELINE config 3's size: a short extrapolation)
        f = max(1, n // 2)
        t0 = time.perf_counter()
        m, bnds = model_and_bounds(n, f, 1, seed)
        t1 = time.perf_counter()
        st, _, _ = oracle_solve(m, relax=True, lb=bnds[0][0], ub=bnds[0][1])
        t_lp = time.perf_counter() - t1
        pts.append((n, f, t_lp, st))
        log(f"cpu baseline: {n}x{f} node LP by HiGHS in {t_lp:.2f}s (status {st})")
        if (time.perf_counter() - t_start) + 4.0 * (time.perf_counter() - t0) > 0.4 * budget:
            break
    xs = np.log([a * a * b for a, b, _, _ in pts[-3:]])
    ys = np.log([t for _, _, t, _ in pts[-3:]])
    p_exp = float(np.polyfit(xs, ys, 1)[0]) if len(pts) >= 2 else 1.0
    n_l, f_l, t_l, _ = pts[-1]
    scale = ((N * N * F) / (n_l * n_l * f_l)) ** p_exp
    # pool throughput at the largest measured size, on the host's per-GPU share of its cores
    w = workers if workers > 0 else cpu_baseline_workers()
    w = max(1, min(w, len(os.sched_getaffinity(0))))
    m, bnds = model_and_bounds(n_l, f_l, w, seed + 1)
    sts, _, wall, w_used = lp_batch_cpu(m, bnds, workers=w)
    pool_lps = len(sts) / wall
    log(f"cpu baseline: {w_used} workers solved {len(sts)} {n_l}x{f_l} node LPs in {wall:.2f}s "
        f"({pool_lps:.2f} LP/s)")
    dnf = _dnf_probe(N, F, seed, fix, max(30.0, budget - (time.perf_counter() - t_start)))
    value = pool_lps / scale
    sample = ("HiGHS (oracle/solve.py, scipy %s) on the reference formulation (oracle/formulation.py), node LPs "
              "with %d c-fixings, same generator. Single-thread times %s; fit t ~ (N^2 F)^%.2f over the last %d "
              "sizes -> %.0f s per %dx%d LP. Pool: %d worker processes solved %d %dx%d LPs in %.2f s = %.2f LP/s; "
              "value = that rate / %.0f (the fitted per-LP time ratio to %dx%d). At %dx%d itself: %s"
              % (__import__("scipy").__version__, fix, ", ".join(f"{a}x{b}: {t:.2f}s" for a, b, t, _ in pts),
                 p_exp, min(3, len(pts)), t_l * scale, N, F, w_used, len(sts), n_l, f_l, wall, pool_lps, scale,
                 N, F, N, F, dnf.get("note", "one node LP solved by HiGHS in %.1f s" % dnf.get("lp_seconds", 0.0))))
    return {"value": value, "unit": "LP-relaxations/s", "cores": w_used, "kind": "port", "sample": sample,
            "host_cpu_count": os.cpu_count(), "affinity_cpu_count": len(os.sched_getaffinity(0)),
            "worker_processes": w_used,
            "cores_note": "one single-threaded HiGHS process per core of this GPU's share of the host "
                          "(host cores / 8 GPUs on a multi-GPU node, capped at the cores this process may use)",
            "extrapolated": True, "pool_lp_per_s_at": {"nodes": n_l, "functions": f_l, "value": pool_lps},
            "dnf_at_bench_size": dnf,
            "measured": [{"nodes": a, "functions": b, "seconds": t, "status": s} for a, b, t, s in pts]}


# the reference's published end-to-end figures for its Alibaba 100x25 trace case (SCIP via OR-Tools 9.6):
# testing/alibaba/alibaba_test/output_<solver>_case0.json "score" and "processing_time" (:7787 / :7800)
ALIBABA_PUBLISHED = {"NeptuneMinDelay": ({"step1": 0.0, "step2": 23.0}, 436.445),
                     "NeptuneMinDelayAndUtilization": ({"step1": 0.005, "step2": 65010.0}, 1258.109),
                     "NeptuneMinUtilization": ({"step1": 1.0, "step2": 65010.0}, 1224.564)}


def alibaba_flows(a):
    """The reference's three Alibaba 100x25 requests (tests/golden/inputs/alibaba_<solver>.json, the payloads of
    testing/alibaba/alibaba_test) through `core.request.solve_request` — the body of main.py's route
    (main.py:31-62): load_data + solve timed as the reference's `processing_time`, step 1 then step 2 (delete,
    then create when delete is not OPTIMAL, neptune.py:18-30) on the GPU engine.  Reported beside the reference's
    recorded score and processing_time; each step's status says whether its B&B proved optimality."""
    from core.request import solve_request
    out = []
    for stype, (ref_score, ref_t) in ALIBABA_PUBLISHED.items():
        with open(os.path.join(REPO, "tests", "golden", "inputs", f"alibaba_{stype}.json")) as fh:
            p = json.load(fh)
        p = json.loads(json.dumps(p))
        p.setdefault("solver", {}).setdefault("args", {})["time_limit"] = a.alibaba_seconds
        p["with_db"] = False
        keep = []
        t0 = time.perf_counter()
        body = solve_request(p, solver_out=keep)
        wall = time.perf_counter() - t0
        s_ = keep[0]
        steps = {}
        for k in ("step1", "step2_delete", "step2_create"):
            r = getattr(getattr(s_, k, None), "result", None)
            if r is not None:
                steps[k] = {"status": r.status, "objective": r.objective, "bound": r.bound, "nodes": r.nodes,
                            "lps": r.lps, "seconds": r.seconds}
        score = {k: float(v) for k, v in body["score"].items()}
        out.append({"solver": stype, "processing_time_s": body["processing_time"], "wall_s": wall,
                    "score": score, "steps": steps,
                    # every step's search ended with a proof: OPTIMAL, or INFEASIBLE (step-2 delete here, after which
                    # the reference falls back to create, neptune.py:24-30)
                    "all_steps_proven": all(v["status"] in ("OPTIMAL", "INFEASIBLE") for v in steps.values() if v),
                    "reference_score": ref_score, "reference_processing_time_s": ref_t,
                    "speedup_vs_reference": ref_t / max(1e-9, body["processing_time"]),
                    "score_matches_reference": all(abs(score[k] - v) <= 1e-6 * max(1.0, abs(v))
                                                   for k, v in ref_score.items())})
        log(f"alibaba {stype}: {body['processing_time']:.2f} s (reference {ref_t:.1f} s), score {score}")
    return out


def bnb_section(a, rank, world, dev, N, F, seconds):
    """The product's own branch-and-bound (core/engine/bnb.py, the search SCIP runs inside
    pywraplp Solve(), solver.py:35-40) on BASELINE config 3's / 4's instance (256x128, 512x256, step-1
    NeptuneMinDelayAndUtilization), time-limited, configured as the product's step 1 runs it
    (NeptuneStepBase.branch_and_bound: facility-relaxation bounds on the branching nodes, reference-model
    leaves, the capacity-greedy root heuristic): node LPs per second INSIDE the B&B, the
    node-LP mix (finished LPs per model/kind and status, iteration percentiles), nodes, incumbent, bound and
    gap.  With N ranks the search is the sharded one (subtrees per rank, one packed all-gather per loop over
    RCCL: core/engine/comm.TorchComm)."""
    from core.engine.comm import LocalComm, TorchComm
    from core.engine.lp import LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    p = synthetic_payload(N, F, seed=a.seed)
    data = data_to_solver_input(p, with_db=False)
    alpha = p["solver"]["args"]["alpha"]
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=alpha, verbose=False, batch=a.batch, lp_tol=a.tol,
                                                lp_max_iters=a.bnb_max_iters)
    st1.load_data(data)
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=a.batch + 2)
    bm = st1.bound_model(data, a.batch + 1)
    comm = TorchComm(device=dev) if world > 1 else LocalComm()
    bnb = st1.branch_and_bound(m, bm, time_limit=seconds, comm=comm, root_max_iters=a.root_max_iters)
    m.reset_stats()
    t0 = time.perf_counter()
    res = bnb.solve()
    wall = time.perf_counter() - t0
    if world > 1:
        wall = comm.max(wall)
    m.close()
    if bm is not None:
        bm.close()
    inc = res.objective
    gap = None if inc is None else (inc - res.bound) / max(1.0, abs(inc))
    d = res.as_dict()
    finished = sum(v for k, v in res.lp_status.items() if k != "presolve_infeasible")
    return {"workload": f"synthetic_{N}x{F}_step1_MDU_product_bnb", "time_limit_s": seconds,
            "status": res.status, "wall_s": wall, "nodes": res.nodes, "leaves": res.leaves, "lps": res.lps,
            "certified_lps": res.certified, "certified_lp_per_s": res.certified / wall, "nodes_per_s": res.nodes / wall,
            "certified_share": res.certified / max(1, finished),
            "resolved_lps": d["resolved"], "resolved_lp_per_s": d["resolved"] / wall,
            "resolved_share": d["resolved"] / max(1, res.lps),
            "lp_status_rank0": res.lp_status, "lp_status_by_kind_rank0": res.lp_status_kind,
            "drained_at_stop": res.drained,
            "lp_iters_p50_p90_p99_max_rank0": d["lp_iters_p50_p90_p99_max"],
            "lp_iterations": res.lp_iterations, "incumbent": inc, "bound": res.bound, "rel_gap": gap,
            "root_seconds": res.timing.get("root"), "host_seconds": {k: res.timing.get(k) for k in
                                                                  ("finish", "submit", "primal", "end")},
            "advance_seconds": res.timing.get("advance"), "ranks": world}


class ReplayStream:
    """The node LPs the product branch-and-bound submitted at this size (recorded by tools/record_bnb_trace.py
    into tests/golden/bnb_trace_<N>x<F>_s<seed>.json.gz), replayed in submission order.  A branching node's box
    is its fixings, a leaf's fixes every c and n (open ones to 1).

    models: {"leaf": (reference LPModel, root slot), "bound": (facility LPModel, root slot) or absent}.
    native=False: every box is an LP relaxation of the REFERENCE model (the LP SCIP solves at that node,
    solver.py:35-40) at the bench's tol / --max-iters, to its certificate.  native=True: every box on the
    model the product ran it on (branching nodes: the facility relaxation) with the product's
    iteration budget, stops (bound_res, gap_tol) and incumbent cutoff — the product's own node-LP mix.
    `batch` slots per model; a node starts from its parent's final PDHG state when a slot of its model still
    holds it (slots are refilled oldest-finished first, as the B&B does; the recorded run's own slot reuse
    is not replayed), else from that model's root.  The
    two roots (depth-0 entries) were solved before the timed region and are skipped.  With `world` ranks,
    rank r takes entries r, r + world, ... (the trace repeated as often as the steps need)."""

    def __init__(self, models, a, rank, world, trace, native=False):
        from collections import Counter, OrderedDict
        self.models, self.a, self.native = models, a, native
        self.lps = [e for e in trace["lps"] if e["parent"] is not None]
        self.parent_of = {e["id"]: e["parent"] for e in trace["lps"]}
        self.ancestors = getattr(a, "warm_ancestors", False)
        self.pos = 0
        self.counter = 0
        self.done = []          # (status, obj, primal_obj, iters) per completed node
        self.kinds = []         # (model, kind) per completed node
        self.depth = []         # (depth, warm from parent) per completed node
        self.where = {}         # (model, node key) -> slot holding its final state
        self.held = {}          # (model, slot) -> node key
        self.running = {}       # (model, slot) -> (node key, kind, depth, warm from parent)
        # `batch` LPs in flight per model, over batch + park slots: a finished node whose children (in this
        # rank's share of the trace) are still to come keeps its slot — its state parked — until its last child
        # started (the oldest parked state is evicted when every slot is taken)
        park = max(0, int(getattr(a, "park", 0)))
        self.free = {name: list(range(a.batch + park)) for name in models}
        self.parked = {name: OrderedDict() for name in models}   # slot -> node key, oldest first
        self.busy = {name: 0 for name in models}
        self.kids = Counter(e["parent"] for e in self.lps)
        self.kids_left = {}     # (model, node key) -> children of it not yet started
        self.warm_parent = 0
        self.records = []       # (--dump) one record per completed node LP
        self.status_of = {}
        # a node is submitted only once its parent's LP finished — as the B&B does (its children exist only
        # then): an entry whose parent still iterates waits (at most 64 such), later ready entries go first
        self.entry_of = {e["id"]: e for e in trace["lps"]}
        self.deferred = []
        self.in_order = bool(getattr(a, "in_order", False))

    def peek_entry(self):
        """(repetition, entry) this rank replays next: the trace's entries in recorded order, once (None at its
        end)."""
        if self.pos >= len(self.lps):
            return None
        return 0, self.lps[self.pos]

    def next_entry(self):
        out = self.peek_entry()
        self.pos += 1
        return out

    def _model(self, e):
        return e["model"] if (self.native and e["model"] in self.models) else "leaf"

    def _box(self, m, e):
        import numpy as np
        F, N = self.a.functions, self.a.nodes
        lb = np.full(m.n_int, -np.inf)
        ub = np.full(m.n_int, np.inf)
        if "open" in e:
            lb[:F * N + N] = ub[:F * N + N] = 0.0
            lb[e["open"]] = ub[e["open"]] = 1.0
        else:
            idx, val = e["fix"]
            lb[idx] = ub[idx] = val
        return lb, ub

    def _candidate(self):
        """(where, rep, entry): the next entry to submit — the first deferred one, else the upcoming one, whose
        parent's LP is not iterating (where = index into `deferred`, -1 = the upcoming entry); None when every
        candidate waits for its parent and the deferral window is full."""
        if self.in_order:
            nxt = self.peek_entry()
            return None if nxt is None else (-1,) + nxt
        running = {(n, v[0]) for (n, _), v in self.running.items()}

        def ready(rep, e):
            pe = self.entry_of.get(e["parent"])
            pm = self._model(pe) if pe is not None else self._model(e)
            return (pm, (rep, e["parent"])) not in running
        for i, (rep, e) in enumerate(self.deferred):
            if ready(rep, e):
                return i, rep, e
        while len(self.deferred) < 64:
            nxt = self.peek_entry()
            if nxt is None:
                return None
            rep, e = nxt
            if ready(rep, e):
                return -1, rep, e
            self.deferred.append(self.next_entry())
        return None

    def _refill(self):
        import math
        from core.engine.lp import LP_INFEASIBLE
        a = self.a
        while self.counter < self.limit:
            cand = self._candidate()
            if cand is None:
                break                            # every candidate waits for its parent's LP
            where_, rep, e = cand
            name = self._model(e)
            if self.busy[name] >= a.batch:
                break                            # the next node waits for a slot of its model
            m, root = self.models[name]
            if self.free[name]:
                slot = self.free[name].pop(0)
            else:                                # every slot parked: evict the oldest parked state
                slot, _ = self.parked[name].popitem(last=False)
            if where_ < 0:
                self.next_entry()
            else:
                del self.deferred[where_]
            key = (rep, e["id"])
            pkey = (name, (rep, e["parent"]))
            old = self.held.pop((name, slot), None)       # this slot's finished state is overwritten now
            if old is not None:
                self.where.pop((name, old), None)
            left = self.kids_left.get(pkey)
            if left is not None:                 # one child of the parent fewer to come: release its slot after the last
                self.kids_left[pkey] = left - 1
                if left - 1 <= 0 and pkey in self.where:
                    ps = self.where[pkey]
                    if self.parked[name].pop(ps, None) is not None:
                        self.free[name].insert(0, ps)
            src = root
            if pkey not in self.where and self.ancestors:
                # (--warm-ancestors: the closest ancestor whose final state a slot still holds)
                p = self.parent_of.get(e["parent"])
                while p is not None and (name, (rep, p)) not in self.where:
                    p = self.parent_of.get(p)
                if p is not None:
                    pkey = (name, (rep, p))
            warm_parent = pkey in self.where
            leaf_start = getattr(a, "leaf_start", "parent") if e["kind"] == "leaf" else "parent"
            if warm_parent and leaf_start == "parent":
                src = self.where[pkey]
                self.warm_parent += 1
            else:
                warm_parent = False
            m.copy_state(src, slot)
            lb, ub = self._box(m, e)
            self.counter += 1
            if self.native:
                kw = dict(max_iters=e["budget"], bound_res=e["bound_res"], gap_tol=e.get("gap_tol", 0.0),
                          cutoff=math.inf if e.get("cutoff") is None else e["cutoff"])
            else:
                kw = dict(max_iters=a.max_iters)
            wf, wc = a.warm_omega_floor, 0.0
            if "open" in e and getattr(a, "leaf_omega", ""):
                wf, wc = (float(t) for t in a.leaf_omega.split(":"))
            st = m.submit([slot], lb[None], ub[None], tol=a.tol, check_every=a.check_every, warm_start=leaf_start != "cold",
                          warm_omega_floor=wf, warm_omega_cap=wc, polish_after=getattr(a, "polish_after", 0.0), **kw)
            if int(st[0]) == LP_INFEASIBLE:
                self.done.append((LP_INFEASIBLE, float("inf"), float("nan"), 0))
                self.kinds.append((name, e["kind"]))
                self.depth.append((e["depth"], warm_parent))
                self.free[name].append(slot)
            else:
                self.running[(name, slot)] = (key, e["kind"], e["depth"], warm_parent)
                self.busy[name] += 1

    def drain(self, n):
        """Stream the next n recorded nodes through the slots until every one of them finished."""
        self.limit = self.counter + n
        self._refill()
        while any(m.active() > 0 for m, _ in self.models.values()):
            for name, (m, _) in self.models.items():
                if m.active() <= 0:
                    continue
                r = m.advance(0 if len(self.models) > 1 else 1)
                for i, slot in enumerate(r["slots"].tolist()):
                    self.done.append((int(r["status"][i]), float(r["obj"][i]), float(r["primal_obj"][i]),
                                      int(r["iters"][i])))
                    key, kind, depth, wp = self.running.pop((name, slot))
                    if getattr(self.a, "dump", None):
                        st_ = int(r["status"][i])
                        rec = {"id": key[1], "kind": kind, "depth": depth, "warm_parent": wp, "status": st_,
                               "iters": int(r["iters"][i]), "parent_status": self.status_of.get(self.parent_of.get(key[1]))}
                        rec["diag"] = m.diag(slot)
                        self.records.append(rec)
                        self.status_of[key[1]] = st_
                    self.busy[name] -= 1
                    self.kinds.append((name, kind))
                    self.depth.append((depth, wp))
                    self.where[(name, key)] = slot
                    self.held[(name, slot)] = key
                    k = self.kids.get(key[1], 0)
                    if k > 0:                    # children to come: park the state
                        self.kids_left[(name, key)] = k
                        self.parked[name][slot] = key
                    else:
                        self.free[name].append(slot)
            self._refill()


def trace_path(a, seed=None):
    seed = a.seed if seed is None else seed
    return os.path.join(REPO, "tests", "golden", f"bnb_trace_{a.nodes}x{a.functions}_s{seed}.json.gz")


def rank_seed(a, rank, world):
    """The instance (generator seed) rank `rank` replays.  One rank: --seed.  N ranks: one recorded B&B per GPU —
    rank r takes seed --seed + r (independent placement requests, weak scaling); without a recorded trace for
    that seed it takes the recorded seeds in turn (tests/golden/bnb_trace_<N>x<F>_s<seed>.json.gz).  The recorded
    512x256 search is one narrow dive (p50 ~25 LPs per depth level, 44 levels): dealing ITS subtrees over 8 ranks
    leaves 56 % of the LPs on one rank (96 % at 2 ranks), so the sharded search itself is measured by the `bnb`
    section (core/engine/bnb.py over RCCL), not by splitting a single-GPU trace."""
    if world <= 1:
        return a.seed
    want = a.seed + rank
    if os.path.exists(trace_path(a, want)):
        return want
    have = [s_ for s_ in range(a.seed, a.seed + 64) if os.path.exists(trace_path(a, s_))]
    return have[rank % len(have)] if have else want


class NodeStream:
    """B&B child LPs of the root, `batch` of them in flight on the engine (nep_lp_submit/advance):
    a slot whose LP finishes takes the next node at once, as a B&B with an open-node queue does."""

    def __init__(self, m, root, a, rank):
        self.m, self.root, self.a, self.rank = m, root, a, rank
        self.counter = 0
        self.done = []          # (status, obj, primal_obj, iters) per completed node

    def _refill(self, slots):
        """Submit the next nodes into the free `slots` (one nep_lp_submit call); stops once `limit`
        nodes were submitted.  Nodes presolve proves infeasible complete at once and their slot
        takes the next node."""
        import numpy as np
        from core.engine.lp import LP_INFEASIBLE
        a = self.a
        free = list(slots)
        while free and self.counter < self.limit:
            take = free[: self.limit - self.counter]
            lbs, ubs = [], []
            for slot in take:
                seed = (a.seed * 1000003 + self.rank) * 7919 + self.counter
                self.counter += 1
                lb, ub = node_bounds(self.m.n_int, a.functions, a.nodes, 1, a.fix, seed)
                lbs.append(lb[0])
                ubs.append(ub[0])
                if not a.cold:
                    self.m.copy_state(self.root, slot)
            st = self.m.submit(take, np.array(lbs), np.array(ubs), tol=a.tol, max_iters=a.max_iters,
                               check_every=a.check_every, warm_start=not a.cold,
                               warm_omega_floor=a.warm_omega_floor)
            free = free[len(take):]
            for slot, code in zip(take, st):
                if int(code) == LP_INFEASIBLE:
                    self.done.append((LP_INFEASIBLE, float("inf"), float("nan"), 0))
                    free.append(slot)

    def drain(self, n):
        """Stream the next n nodes through the `batch` slots until every one of them finished."""
        self.limit = self.counter + n
        self._refill(range(self.a.batch))
        while self.m.active() > 0:
            r = self.m.advance(1)
            for i in range(len(r["slots"])):
                self.done.append((int(r["status"][i]), float(r["obj"][i]), float(r["primal_obj"][i]),
                                  int(r["iters"][i])))
            self._refill(r["slots"].tolist())


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        return s_.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus n` > 1 without a launcher: start n rank processes (torch.distributed.run, one per GPU, rendezvous
    on 127.0.0.1) running this script with the same arguments, as a CHILD process — this process has not
    touched the GPU and never replaces itself — and return their exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd)


def rank_world(a):
    """(rank, world, local rank) of this process.  The world a launcher started must be the one --gpus asks
    for: a mismatch fails instead of measuring a different number of GPUs than the JSON line would claim."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    return rank, world, local


def _probe_ranks(a, rank, world):
    """NEP_BENCH_PROBE_RANKS=k (CPU tests, tests/test_bench_launch.py): join a gloo group, print this rank's
    first k replay entries (ReplayStream's rank, rank + world, ... split) and exit before any GPU work."""
    import gzip
    import torch.distributed as td
    td.init_process_group("gloo")
    seed = rank_seed(a, rank, world)
    with gzip.open(trace_path(a, seed), "rt") as fh:
        trace = json.load(fh)
    rs = ReplayStream({}, a, rank, world, trace)
    ids = [rs.next_entry()[1]["id"] for _ in range(int(os.environ["NEP_BENCH_PROBE_RANKS"]))]
    got = [None] * world
    td.all_gather_object(got, {"rank": rank, "world": world, "seed": seed, "ids": ids, "entries": len(rs.lps)})
    if rank == 0:
        print(json.dumps({"probe": "ranks", "ranks": got, "n_gpus": world}), flush=True)
    td.destroy_process_group()


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    rank, world, local = rank_world(a)
    if os.environ.get("NEP_BENCH_PROBE_RANKS"):
        return _probe_ranks(a, rank, world)
    import numpy as np
    import torch

    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as td
        td.init_process_group("nccl", device_id=dev)

    from core.engine.lp import LPModel, LP_BOUND, LP_CUTOFF, LP_INFEASIBLE, LP_ITERATION_LIMIT, LP_OPTIMAL
    STATUS_NAME = {LP_OPTIMAL: "certified", LP_ITERATION_LIMIT: "limit", LP_INFEASIBLE: "infeasible",
                   LP_CUTOFF: "cutoff", LP_BOUND: "bound"}
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload

    N, F, B = a.nodes, a.functions, a.batch
    seed = rank_seed(a, rank, world)
    payload = synthetic_payload(N, F, seed=seed)
    data = data_to_solver_input(payload, with_db=False)
    alpha = payload["solver"]["args"]["alpha"]
    park = max(0, a.park)
    root = B + park          # (slots 0 .. B + park - 1: the streams' working and parking slots)
    t_build = time.perf_counter()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=root + 1)
    log(f"rank {rank}: model {N}x{F}: R={m.info.n_rows} rows, P={m.info.x_entries} routing entries, "
        f"built in {time.perf_counter() - t_build:.1f}s")
    P = m.info.x_entries
    t_root = time.perf_counter()
    rr = m.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every,
                 polish_after=float(a.root_polish_after))
    root_obj, root_status, root_iters = float(rr["obj"][0]), int(rr["status"][0]), int(rr["iters"][0])
    root_seconds = time.perf_counter() - t_root
    root_omega = m.diag(root)["omega"]
    if a.omega_ref > 0:
        m.set_reference_weight(a.omega_ref * m.info.primal_weight0)
    log(f"rank {rank}: root LP status {root_status} obj {root_obj:.10g} after {root_iters} iterations "
        f"({time.perf_counter() - t_root:.2f}s)")
    if root_status != LP_OPTIMAL:
        raise RuntimeError(f"root LP not certified: status {root_status} after {root_iters} iterations")
    root_polish = None
    if a.root_gap_tol > 0:
        # the children's starting point: the root's state continued to a tighter objective gap (the
        # certified root value above stands; the polished state is kept whether or not it certifies)
        t_pol = time.perf_counter()
        rp = m.solve([root], tol=a.tol, gap_tol=a.root_gap_tol, max_iters=a.root_max_iters,
                     check_every=a.root_check_every, warm_start=True, warm_omega_floor=-1.0)
        root_polish = {"gap_tol": a.root_gap_tol, "status": int(rp["status"][0]), "iters": int(rp["iters"][0]),
                       "obj": float(rp["obj"][0]), "seconds": time.perf_counter() - t_pol}
        log(f"rank {rank}: root polish to gap {a.root_gap_tol:g}: status {root_polish['status']} after "
            f"{root_polish['iters']} iterations ({root_polish['seconds']:.2f}s)")

    kind = a.stream
    if kind == "auto":
        kind = "replay" if os.path.exists(trace_path(a, seed)) else "children"
    bm = fac_root = None
    if kind == "replay":
        import gzip
        with gzip.open(trace_path(a, seed), "rt") as fh:
            trace = json.load(fh)
        stream = ReplayStream({"leaf": (m, root)}, a, rank, world, trace)
        if a.native_steps > 0:
            # the facility relaxation (the product's bound model) and its root, stopped as the product's is:
            # bound converged (bound_res 1e-2, gap_tol 1e-4) or the root budget (core/engine/bnb.py _submit)
            from core.engine.lp import RELAX_FACILITY
            bm = LPModel(data, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=root + 1,
                         relaxation=RELAX_FACILITY)
            t_fr = time.perf_counter()
            fr = bm.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every,
                        bound_res=1e-2, gap_tol=1e-4)
            # (the facility model keeps the parent-relative warm-start band, as in the product search)
            fac_root = {"status": int(fr["status"][0]), "obj": float(fr["obj"][0]), "iters": int(fr["iters"][0]),
                        "seconds": time.perf_counter() - t_fr}
            log(f"rank {rank}: facility-relaxation root: {fac_root}")
    else:
        stream = NodeStream(m, root, a, rank)

    def timed(stream, steps, tag, count=None):
        """steps * B nodes of `stream` (or `count` of them), drained, timed between barriers (max over ranks)."""
        m.reset_stats()
        if bm is not None:
            bm.reset_stats()
        i0 = len(stream.done)
        if dist:
            td.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # the timed K steps: K*B nodes (the replay: the whole recorded trace, K steps of 1/K of it each) streamed
        # through the B slots and drained (every node finished, hard ones included — no node is left iterating
        # outside the timed region)
        stream.drain(steps * B if count is None else count)
        ok = [o for st_, o, _, _ in stream.done[i0:] if st_ == LP_OPTIMAL]
        best = torch.tensor([min(ok) if ok else float("inf")], dtype=torch.float64, device=dev)
        if dist:
            td.all_reduce(best, op=td.ReduceOp.MIN)     # B&B bound exchange (8 B)
        torch.cuda.synchronize()
        if dist:
            td.barrier()
        wall = time.perf_counter() - t0
        log(f"rank {rank}: {tag}: {len(stream.done) - i0} node LPs completed in {wall:.2f}s")
        res = stream.done[i0:]
        n_ok = sum(1 for r in res if r[0] == LP_OPTIMAL)
        n_first = sum(1 for r in res if r[0] == LP_OPTIMAL and r[3] <= 1)
        n_res = sum(1 for r in res if r[0] in (LP_OPTIMAL, LP_INFEASIBLE, LP_BOUND, LP_CUTOFF))
        n_it = sum(r[3] for r in res)
        gmax = max([abs(p_ - o) / max(1.0, abs(o)) for s_, o, p_, _ in res if s_ == LP_OPTIMAL] or [0.0])
        st = m.stats()
        util = n_it / max(1, st["lp_iterations"])       # this rank's LP iterations / slot-iterations run
        iq = [int(v) for v in np.percentile([r[3] for r in res], [50, 90, 100])] if res else [0, 0, 0]
        split = None
        dep = getattr(stream, "depth", None)
        if dep is not None and len(dep) >= len(stream.done):
            # iterations per node LP by warm-start source (parent's parked state vs the root's) and by depth
            dd = dep[i0:]
            split = {}
            for tag, sel in (("parent", lambda d_, w_: w_), ("root", lambda d_, w_: not w_)):
                its = [r[3] for r, (d_, w_) in zip(res, dd) if sel(d_, w_)]
                ok_ = [r[0] == LP_OPTIMAL for r, (d_, w_) in zip(res, dd) if sel(d_, w_)]
                split[tag] = {"lps": len(its), "mean_iters": float(np.mean(its)) if its else None,
                              "certified_share": float(np.mean(ok_)) if ok_ else None}
            for lo_, hi_ in ((0, 10), (10, 20), (20, 30), (30, 1000)):
                for tag in ("parent", "root"):
                    its = [r[3] for r, (d_, w_) in zip(res, dd) if lo_ <= d_ < hi_ and w_ == (tag == "parent")]
                    split[f"depth{lo_}-{hi_ - 1}_{tag}"] = ({"lps": len(its), "mean_iters": float(np.mean(its))}
                                                           if its else None)
        tot = torch.tensor([wall, n_ok, n_it, gmax, len(res), n_first, n_res], dtype=torch.float64, device=dev)
        if dist:
            mx = tot.clone()
            td.all_reduce(mx, op=td.ReduceOp.MAX)
            sm = tot.clone()
            td.all_reduce(sm, op=td.ReduceOp.SUM)
            tot = torch.cat([mx[:1], sm[1:3], mx[3:4], sm[4:]])
        wall, n_ok, n_it, gmax, n_done, n_first, n_res = (float(t) for t in tot.tolist())
        return {"wall": wall, "certified": int(n_ok), "completed": int(n_done), "iterations": int(n_it),
                "gmax": gmax, "first_check_certified": int(n_first), "resolved": int(n_res), "iters_p50_p90_max": iq,
                "util": util, "stats": st, "warm_split_rank0": split}

    if a.warmup > 0:
        # untimed: the first W x B boxes (replay: on a stream of their own — the timed region then replays the
        # whole trace from its start, so `value` does not depend on --steps / --warmup)
        ws = ReplayStream({"leaf": (m, root)}, a, rank, world, trace) if kind == "replay" else stream
        ws.drain(a.warmup * B)
        log(f"rank {rank}: warmup: {len(ws.done)} node LPs completed")
    prim = timed(stream, a.steps, kind, count=len(stream.lps) if kind == "replay" else None)
    if a.dump and rank == 0 and getattr(stream, "records", None) is not None:
        with open(a.dump, "w") as fh:
            json.dump(stream.records, fh)
    st = prim["stats"]
    wall, n_ok, n_it, gmax, n_done = prim["wall"], prim["certified"], prim["iterations"], prim["gmax"], prim["completed"]
    iq, util = prim["iters_p50_p90_max"], prim["util"]
    second = native = None
    if kind == "replay" and bm is not None:
        # the product's own node-LP mix: every recorded box on the model the B&B ran it on, with its budget,
        # stops and cutoff (branching nodes: the facility relaxation; leaves: the reference model)
        ns = ReplayStream({"leaf": (m, root), "bound": (bm, root)}, a, rank, world, trace, native=True)
        nat = timed(ns, a.native_steps, "replay (native models)")
        mix = {}
        for (name, k), r in zip(ns.kinds, ns.done):
            d = mix.setdefault(f"{name}/{k}", {})
            s_ = STATUS_NAME.get(r[0], str(r[0]))
            d[s_] = d.get(s_, 0) + 1
        native = {"workload": workload_name(a, "replay") + "_native_models", "resolved_lp_per_s":
                  nat["resolved"] / nat["wall"], "certified_lp_per_s": nat["certified"] / nat["wall"],
                  "resolved": nat["resolved"], "certified": nat["certified"], "completed": nat["completed"],
                  "steps": a.native_steps, "wall_s": nat["wall"], "iters_p50_p90_max": nat["iters_p50_p90_max"],
                  "status_by_model_kind_rank0": mix, "facility_root": fac_root,
                  "note": "resolved = certified + infeasible + cutoff + bound-converged (LP_BOUND); branching "
                          "nodes that end at their 1024-iteration budget keep a valid bound but are not counted"}
        bm.close()
    if kind == "replay" and a.children_steps > 0:
        # the secondary figure: the round-1..3 stream of root children with 2 random c-fixings each
        cs = NodeStream(m, root, a, rank)
        sec = timed(cs, a.children_steps, "children")
        second = {"workload": children_workload_name(a), "value": sec["certified"] / sec["wall"],
                  "certified": sec["certified"], "completed": sec["completed"], "steps": a.children_steps,
                  "wall_s": sec["wall"], "iters_p50_p90_max": sec["iters_p50_p90_max"],
                  "first_check_certified_share": sec["first_check_certified"] / max(1, sec["completed"])}
    m.close()
    # the product's own B&B (every rank takes part: the sharded search when world > 1)
    bnb = None
    if a.bnb_seconds > 0:
        bnb = []
        for size in a.bnb_sizes.split(","):
            size, _, secs = size.partition(":")
            bn, bf = (int(t) for t in size.lower().split("x"))
            bnb.append(bnb_section(a, rank, world, dev, bn, bf, float(secs) if secs else a.bnb_seconds))
            log(f"rank {rank}: bnb {size}: {bnb[-1]['certified_lps']} certified node LPs, status {bnb[-1]['status']}, "
                f"gap {bnb[-1]['rel_gap']}")
    if rank != 0:
        if dist:
            td.destroy_process_group()
        return

    # algorithmic bytes of one PDHG iteration of one LP: SURVEY.md §8(d) B_iter = 4 (2P + 2FN + 2N + 2m),
    # x read + write, c and n read + write, duals read + write (fp32 units), P = R x N routing entries
    # after exact aggregation, m = the dualised rows (nep_model_info.bytes_per_iter)
    per_lp = float(m.info.bytes_per_iter)
    launch_ms = st["x_pass_ms"] / max(1, st["x_pass_sampled"])
    lps_per_launch = st["x_pass_lp_iters"] / max(1, st["x_pass_sampled"])
    achieved = per_lp * lps_per_launch / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    workload = workload_name(a, kind)
    traffic = traffic_ratio = None
    if os.path.exists(a.traffic):
        with open(a.traffic) as fh:
            t = json.load(fh)
        if t.get("workload") == workload:
            # measured per LP-iteration (PMC passes at t["lps_per_launch"] slots), scaled to the LPs
            # of this run's average sampled launch so it compares with `achieved`'s bytes
            per_lp_iter = t["bytes_per_launch"] / max(1, t.get("lps_per_launch", 1))
            traffic = per_lp_iter * lps_per_launch
            traffic_ratio = per_lp_iter / per_lp
    flows = alibaba_flows(a) if (world == 1 and a.alibaba_seconds > 0) else None
    cpu = None
    if world == 1 and a.cpu_budget > 0:
        cpu = cpu_baseline(N, F, a.seed, a.fix, a.cpu_budget, a.cpu_workers)
    out = {
        "metric": "LP-relaxations/sec + objective gap vs reference, 512-node×256-function",
        "value": n_ok / wall,
        "unit": "LP-relaxations/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": wall / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 x-state, f64 duals/reductions/certificate",
        "data": "synthetic (SURVEY.md §8(d) generator, seed %d)" % a.seed,
        "config": {"workload": workload, "nodes": N, "functions": F, "lp_in_flight_per_gpu": B,
                   "fixings_per_lp": a.fix if kind == "children" else "recorded B&B boxes", "tol": a.tol, "max_iters_per_lp": a.max_iters,
                   "routing_entries_P": P,
                   "parallelism": (f"bnb-subtrees x{world}" if kind != "replay" else
                                   ("one recorded B&B" if world == 1 else f"one recorded B&B per GPU x{world}")),
                   "timed_lps_per_rank": (len(stream.lps) if kind == "replay" else a.steps * B),
                   "instance_seed_rank0": seed,
                   "workload_note": ("value = certified LP relaxations of the REFERENCE model (the LP SCIP solves at "
                                     "each node) at the boxes the product's own 512x256 B&B submitted in 60 s "
                                     "(tests/golden/bnb_trace_512x256_s<seed>.json.gz), the whole trace once per "
                                     "rank in recorded order (a box waits for its parent's LP; finished parents "
                                     "park their state, --park slots); one step = 1/K of the trace.  The product "
                                     "search's own node-LP rate (branching nodes on the facility relaxation, "
                                     "budgets, stops) is `product_node_lp_per_s`"
                                     if kind == "replay" else "root children with random c-fixings")},
        "product_node_lp_per_s": {
            "native_replay_resolved": native["resolved_lp_per_s"] if native else None,
            "native_replay_certified": native["certified_lp_per_s"] if native else None,
            "bnb_resolved": ({b_["workload"]: b_["resolved_lp_per_s"] for b_ in bnb} if bnb else None),
            "bnb_certified": ({b_["workload"]: b_["certified_lp_per_s"] for b_ in bnb} if bnb else None),
            "note": "the product B&B's node LPs per second: resolved = certified + bound-converged + proven "
                    "infeasible + cut off (every such LP ends its node); native_replay = the trace's first "
                    "boxes on the models the product ran them on; bnb = the product search itself"},
        "alibaba_flows": flows,
        "objective_gap": {"certified_max": gmax, "tol": a.tol,
                          "note": "(primal obj - Lagrangian bound)/max(1,|bound|) per certified LP; "
                                  "HiGHS parity on the reference's own models: tests/test_gpu_lp.py"},
        "lp": {"stream": kind, "certified": n_ok, "completed": n_done, "iterations": n_it,
               "resolved": prim["resolved"], "resolved_lp_per_s": prim["resolved"] / wall,
               "first_check_certified_share": prim["first_check_certified"] / max(1, n_done),
               "warm_from_parent_rank0": getattr(stream, "warm_parent", None),
               "park_slots": a.park, "iters_by_warm_source_rank0": prim["warm_split_rank0"],
               "mean_iters": n_it / max(1, n_done), "iters_p50_p90_max": iq,
               "slot_utilisation_rank0": util,
               "root_obj": root_obj, "root_iters": root_iters, "root_seconds": root_seconds,
               "primal_weight0": m.info.primal_weight0, "root_final_weight": root_omega,
               "omega_ref": a.omega_ref * m.info.primal_weight0 if a.omega_ref > 0 else None,
               "root_polish": root_polish},
        "native_replay": native,
        "children_stream": second,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_over_algorithmic": traffic_ratio,
                     "kernel": "x_pass", "algorithmic_bytes_per_launch": per_lp * lps_per_launch,
                     "algorithmic_bytes_per_lp_iter": per_lp,
                     "algorithmic_formula": "SURVEY.md 8(d) B_iter = 4(2P + 2FN + 2N + 2m), P = R*N, m = dualised rows",
                     "avg_launch_ms": launch_ms, "sampled_launches": st["x_pass_sampled"]},
        "cpu_baseline": cpu,
        "bnb": bnb,
    }
    print(json.dumps(out), flush=True)
    if dist:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
