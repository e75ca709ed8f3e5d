#!/usr/bin/env python3
"""HBM traffic of the bench's dominant kernel (x_pass) from rocprofv3 PMC counters.

On the GPU box, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 tools/traffic.py run
  rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 tools/traffic.py run
Then (anywhere):
  python3 tools/traffic.py summarize gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/traffic.json

`run` builds bench.py's default model (same generator, seed, batch), solves its root LP, starts `batch`
node LPs on the first boxes of the bench's replay stream (tests/golden/bnb_trace_*.json.gz) warm from the
root's state as the replay does, and runs 4 blocks of PDHG iterations: x_pass steady-state launches with all
`batch` LPs active, as in the bench's timed region (`run cold`: no root solve, the nodes cold — the round-4
workaround for the SIGSEGV of the first --pmc pass, DESIGN.md §6 "PMC pass crash").  `summarize` averages the counters
over the steady-state x_pass launches (x_pass<CPL, false, false>, full grid) and converts them:
FETCH_SIZE and WRITE_SIZE are KiB (rocprofiler-sdk derived_counters.xml); FETCH_SIZE is doubled for
wide streaming reads on gfx950 (MI355X_MICROARCH.md, HBM).
"""
import json
import os
import sqlite3
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]


def run():
    import numpy as np
    import bench
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    import gzip
    a = bench.parse([])
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    cold = len(sys.argv) > 2 and sys.argv[2] == "cold"
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=a.batch + 1)
    root = a.batch
    if not cold:
        m.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every)
    with gzip.open(bench.trace_path(a), "rt") as fh:
        trace = json.load(fh)
    rs = bench.ReplayStream({"leaf": (m, root)}, a, 0, 1, trace)
    boxes = [rs._box(m, e) for e in rs.lps[:a.batch]]
    lb = np.array([b[0] for b in boxes])
    ub = np.array([b[1] for b in boxes])
    if not cold:
        for s in range(a.batch):
            m.copy_state(root, s)
    m.submit(np.arange(a.batch), lb, ub, tol=a.tol, max_iters=a.max_iters, check_every=a.check_every,
             warm_start=not cold)
    for _ in range(4):
        m.advance(0)
    print(json.dumps({"workload": bench.workload_name(a, "replay"), "active": m.active(), "P": m.info.x_entries}))
    m.close()


def _counters(d, F):
    """Per-launch counter values of the steady-state x_pass launches, keyed by (counter, LP slots in
    the launch); slots = workgroups / F (the x-pass grid is F x slots workgroups, padded to a
    multiple of 8 for its XCD-aware order)."""
    dbs = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith(".db")]
    vals = {}
    for db in dbs:
        c = sqlite3.connect(db)
        q = ("select k.name, k.grid_x * k.grid_y / k.workgroup_x, p.counter_name, p.value from counters_collection p "
             "join kernels k on k.dispatch_id = p.dispatch_id")
        for name, wgs, cname, v in c.execute(q):
            if "x_pass" in name and "false, false, false" in name:   # steady state: not CHECK/INIT/FIRST
                vals.setdefault((cname, int(wgs) // F), []).append(float(v))
    return vals


def summarize(fetch_dir, write_dir):
    import bench
    a = bench.parse([])
    f = _counters(fetch_dir, a.functions)
    w = _counters(write_dir, a.functions)
    fk = max(f, key=lambda k: (k[1], len(f[k])))
    wk = max(w, key=lambda k: (k[1], len(w[k])))
    fetch_kib = sum(f[fk]) / len(f[fk])
    write_kib = sum(w[wk]) / len(w[wk])
    fetch_b = 2.0 * fetch_kib * 1024.0
    write_b = write_kib * 1024.0
    out = {"workload": bench.workload_name(a, "replay"), "kernel": "x_pass<CPL,false,false>", "lps_per_launch": fk[1],
           "fetch_kib_raw": fetch_kib, "write_kib_raw": write_kib, "fetch_bytes": fetch_b, "write_bytes": write_b,
           "bytes_per_launch": fetch_b + write_b, "launches": [len(f[fk]), len(w[wk])],
           "note": "FETCH_SIZE x2 (gfx950 wide-read tally), KiB -> bytes; per steady-state x_pass launch; the bench model with the replay stream's first `batch` boxes iterating"}
    print(json.dumps(out, indent=1))


def summarize_sq(d):
    """Average of every counter of one PMC pass (e.g. the SQ_* issue / wait counters) over the
    steady-state x_pass launches with the most LP slots."""
    import bench
    a = bench.parse([])
    c = _counters(d, a.functions)
    top = max(k[1] for k in c)
    out = {"workload": bench.workload_name(a, "replay"), "kernel": "x_pass<CPL,false,false,false>", "lps_per_launch": top,
           "counters": {k[0]: sum(v) / len(v) for k, v in c.items() if k[1] == top},
           "launches": max(len(v) for k, v in c.items() if k[1] == top)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    elif sys.argv[1] == "sq":
        summarize_sq(sys.argv[2])
    else:
        summarize(sys.argv[2], sys.argv[3])
