#!/usr/bin/env python3
"""Dev-only: the numpy mirror of the engine (tests/ref_pdhg.py) over every golden LP case (root +
node fixings), against the HiGHS values — the CPU twin of tests/test_gpu_lp.py, for iterating on
the algorithm without a GPU.  Prints one line per LP and a summary."""
import sys
import time

sys.path[:0] = ["/root/repo/neptune-mip_amd", "/root/repo", "/root/repo/tests"]
import numpy as np  # noqa: E402
import ref_pdhg  # noqa: E402
from gpu_cases import G, build_args, fixing_bounds, lp_cases  # noqa: E402

tol = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-7
max_iters = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
only = sys.argv[3] if len(sys.argv) > 3 else None
bad = tot = 0
its = []
t0 = time.time()
for name, k in lp_cases():
    if only and only not in name:
        continue
    data, variant, step, kw = build_args(name, k)
    m = ref_pdhg.RefModel(data, variant, step, **kw)
    N, F = len(data.nodes), len(data.functions)
    nodes = [(None, None, G[name]["models"][k]["lp_objective"])] + fixing_bounds(name, k, m.n_int, N * N * F)
    for b, (lb, ub, ref) in enumerate(nodes):
        r = ref_pdhg.solve(m, lb, ub, tol=tol, max_iters=max_iters)
        tot += 1
        if ref is None:
            ok = r["status"] != 0
        else:
            ok = r["status"] == 0 and abs(r["obj"] - ref) <= 1e-6 * max(1.0, abs(ref))
        its.append(r["iters"])
        if not ok:
            bad += 1
            print(f"BAD {name}__{k} node{b} st={r['status']} it={r['iters']} obj={r['obj']:.10g} ref={ref}",
                  flush=True)
print(f"bad {bad}/{tot}  iters median {np.median(its):.0f} max {max(its)}  {time.time() - t0:.0f}s")
