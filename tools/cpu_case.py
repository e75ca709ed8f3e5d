#!/usr/bin/env python3
"""Dev-only: run the numpy mirror of the engine (tests/ref_pdhg.py) on one golden model, verbose."""
import sys

sys.path[:0] = ["/root/repo/neptune-mip_amd", "/root/repo", "/root/repo/tests"]
import ref_pdhg  # noqa: E402
from gpu_cases import G, build_args  # noqa: E402

name, k = sys.argv[1], int(sys.argv[2])
data, variant, step, kw = build_args(name, k)
m = ref_pdhg.RefModel(data, variant, step, **kw)
print("omega0", m.omega0, "ref", G[name]["models"][k]["lp_objective"])
r = ref_pdhg.solve(m, tol=1e-7, max_iters=int(sys.argv[3]) if len(sys.argv) > 3 else 100000, verbose=True)
print("status", r["status"], "obj", r["obj"], "iters", r["iters"])
