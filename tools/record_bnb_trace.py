#!/usr/bin/env python3
"""Record the node LPs the product branch-and-bound submits (core/engine/bnb.py trace=) on a synthetic
instance, for bench.py's replay stream (tests/golden/bnb_trace_<N>x<F>_s<seed>.json.gz).  Runs on the GPU box;
the search is the product's (facility-relaxation bounds, reference-model leaves), time-limited.

  python3 tools/record_bnb_trace.py 512 256 60 gpurun_out/trace     [seed 0]
"""
import gzip
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]


def main():
    from core.engine.lp import LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F, secs, out = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
    seed = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    p = synthetic_payload(N, F, seed=seed)
    data = data_to_solver_input(p, with_db=False)
    # the product's step-1 search (NeptuneStepBase.branch_and_bound) at bench.py's defaults: 32 node LPs in
    # flight per model, tol 1e-6, 4096-iteration leaves (branching nodes a quarter of that)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6, lp_max_iters=4096)
    st1.load_data(data)
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    bm = st1.bound_model(data, 33)
    trace = []
    t0 = time.time()
    try:
        res = st1.branch_and_bound(m, bm, time_limit=secs, root_max_iters=400000, trace=trace).solve()
    finally:
        m.close()
        bm.close()
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, f"bnb_trace_{N}x{F}_s{seed}.json.gz")
    doc = {"nodes": N, "functions": F, "seed": seed, "seconds": time.time() - t0, "status": res.status,
           "incumbent": res.objective, "bound": res.bound, "generator": "tools/record_bnb_trace.py",
           "lps": trace}
    with gzip.open(path, "wt", compresslevel=9) as fh:
        json.dump(doc, fh, separators=(",", ":"))
    kinds = {}
    for e in trace:
        kinds[e["kind"]] = kinds.get(e["kind"], 0) + 1
    print(f"{N}x{F}: {len(trace)} LPs {kinds}, status {res.status}, incumbent {res.objective}, bound {res.bound} "
          f"-> {path} ({os.path.getsize(path)} B)", flush=True)


if __name__ == "__main__":
    main()
