#!/usr/bin/env python3
"""Dev probe (GPU box): does the product's step-1 search close (round-5 VERDICT #1)?  Runs
NeptuneStep1CPUMinDelayAndUtilization's two-model search (facility-relaxation branching nodes, reference-model
leaves, native tree) on SURVEY §8(d) instances with a time limit, per branching rule, and prints one JSON line per
run: status, incumbent, bound, relative gap, nodes, LPs, seconds — beside the optimum HiGHS 1.8 proved on the
same instance's aggregated facility MIP on this container's CPU (the facility rows with C2's eps floor, exact for
integral c / n; /tmp experiment, DESIGN.md §7 "Closing the search").

  python3 tools/bnb_close_probe.py 48x24:60,64x32:120 [--rules 0,1] [--gap 1e-4] [--seed 0] [--out f.jsonl]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

# HiGHS 1.8 (scipy milp) on the aggregated facility MIP of synthetic_payload(N, F, seed=0), alpha 0.5: proven optima
HIGHS_OPT = {"48x24": (0.13311272039486574, 4.3), "56x28": (0.13542872678750384, 132.3),
             "64x32": (0.13592086575599188, 482.8)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sizes")
    ap.add_argument("--rules", default="0,1")
    ap.add_argument("--gap", type=float, default=1e-4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--node-iters", type=int, default=0)
    ap.add_argument("--bound-gap", type=float, default=0.0)
    ap.add_argument("--node-limit", type=float, default=1e9)
    ap.add_argument("--strong-iters", type=int, default=256)
    ap.add_argument("--strong-cands", type=int, default=8)
    ap.add_argument("--tag", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from core.engine.lp import LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    rows = []
    for item in a.sizes.replace("+", ",").split(","):
        size, _, secs = item.partition(":")
        N, F = (int(t) for t in size.split("x"))
        data = data_to_solver_input(synthetic_payload(N, F, seed=a.seed), with_db=False)
        for rule in (int(r) for r in a.rules.replace("+", ",").split(",")):
            st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=a.batch, lp_tol=1e-6,
                                                        lp_max_iters=4096)
            st1.load_data(data)
            m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=a.batch + 2)
            bm = st1.bound_model(data, a.batch + 1)
            ov = dict(time_limit=float(secs or 60), root_max_iters=400000, gap=a.gap, branching=rule,
                      node_limit=a.node_limit, strong_iters=a.strong_iters, strong_cands=a.strong_cands)
            if a.node_iters:
                ov["node_max_iters"] = a.node_iters
            if a.bound_gap:
                ov["bound_gap"] = a.bound_gap
            t0 = time.time()
            try:
                res = st1.branch_and_bound(m, bm, **ov).solve()
            finally:
                m.close()
                bm.close()
            inc = res.objective
            ref = HIGHS_OPT.get(size) if a.seed == 0 else None
            row = {"instance": size, "seed": a.seed, "rule": rule, "tag": a.tag, "node_iters": a.node_iters,
                   "bound_gap": a.bound_gap, "time_limit": float(secs or 60), "status": res.status, "strong": res.strong,
                   "incumbent": inc, "bound": res.bound,
                   "rel_gap": None if inc is None else (inc - res.bound) / max(1.0, abs(inc)),
                   "nodes": res.nodes, "lps": res.lps, "seconds": time.time() - t0, "native": res.native,
                   "highs_optimum": ref[0] if ref else None, "highs_seconds": ref[1] if ref else None,
                   "lp_status_kind": res.lp_status_kind}
            print(json.dumps(row), flush=True)
            rows.append(row)
    if a.out:
        with open(a.out, "w") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
