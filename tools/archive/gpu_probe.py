#!/usr/bin/env python3
"""Diagnostics for one gpurun call: solve every golden LP case on the GPU, print one line each."""
import sys, time, traceback
sys.path[:0] = ["/root/repo/neptune-mip_amd", "/root/repo", "/root/repo/tests"]
import numpy as np
from gpu_cases import G, build_args, fixing_bounds, lp_cases
from core.engine.lp import LPModel

bad = 0
for name, k in lp_cases():
    try:
        data, variant, step, kw = build_args(name, k)
        rec = G[name]["models"][k]
        N, F = len(data.nodes), len(data.functions)
        m0 = None
        nodes = G[name]['models'][k].get('node_lps', [])
        m = LPModel(data, variant, step=step, max_batch=1 + len(nodes), **kw)
        nodes = fixing_bounds(name, k, m.n_int, N * N * F)
        B = 1 + len(nodes)
        lb = np.full((B, m.n_int), -np.inf); ub = np.full((B, m.n_int), np.inf)
        for b, (l, u, _) in enumerate(nodes):
            lb[b + 1], ub[b + 1] = l, u
        t = time.time()
        res = m.solve(np.arange(B), lb, ub, max_iters=int(sys.argv[1]) if len(sys.argv) > 1 else 20000)
        dt = time.time() - t
        refs = [rec["lp_objective"]] + [r for _, _, r in nodes]
        for b, ref in enumerate(refs):
            obj = res["obj"][b]
            ok = (ref is None and res["status"][b] != 0) or (ref is not None and res["status"][b] == 0 and abs(obj - ref) <= 1e-6 * max(1, abs(ref)))
            bad += not ok
            print(f"{'OK ' if ok else 'BAD'} {name}__{k} node{b} st={res['status'][b]} it={res['iters'][b]} obj={obj:.9g} "
                  f"p={res['primal_obj'][b]:.9g} ref={ref} ({dt:.2f}s)", flush=True)
        m.close()
    except Exception:
        bad += 1
        print("EXC", name, k, traceback.format_exc(), flush=True)
print("BAD", bad)
