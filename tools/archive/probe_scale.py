#!/usr/bin/env python3
"""Dev probe (GPU box): root-LP and warm-started child LPs of the synthetic generator at growing
sizes; prints iterations, status, wall time and the sampled x-pass bandwidth per size."""
import sys
import time

sys.path[:0] = ["/root/repo/neptune-mip_amd", "/root/repo"]
import numpy as np  # noqa: E402

from core.engine.lp import LPModel  # noqa: E402
from core.utils import data_to_solver_input  # noqa: E402
from core.utils.synthetic import synthetic_payload  # noqa: E402
from bench import node_bounds  # noqa: E402

sizes = [tuple(map(int, s.split("x"))) for s in (sys.argv[1:] or ["64x32", "256x128", "512x256"])]
for N, F in sizes:
    p = synthetic_payload(N, F, seed=0)
    d = data_to_solver_input(p, with_db=False)
    B = 8
    t = time.time()
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=B + 1)
    tb = time.time() - t
    t = time.time()
    r = m.solve([B], tol=1e-6, max_iters=int(__import__("os").environ.get("PROBE_MAX_ITERS", "60000")))
    tr = time.time() - t
    s = m.stats()
    bw = 8.0 * m.info.x_entries * s["x_pass_lp_iters"] / max(1e-9, s["x_pass_ms"] * 1e-3) / 1e9
    print(f"{N}x{F}: R={m.info.n_rows} P={m.info.x_entries} build {tb:.1f}s | root st={r['status'][0]} "
          f"it={r['iters'][0]} obj={r['obj'][0]:.10g} p={r['primal_obj'][0]:.10g} {tr:.2f}s "
          f"x_pass {s['x_pass_ms'] / max(1, s['x_pass_sampled']):.4f} ms/launch ~{bw:.0f} GB/s", flush=True)
    print("   diag", m.diag(B), flush=True)
    m.reset_stats()
    lb, ub = node_bounds(m.n_int, F, N, B, 2, seed=1)
    for b in range(B):
        m.copy_state(B, b)
    t = time.time()
    r = m.solve(np.arange(B), lb, ub, tol=1e-6, max_iters=int(__import__("os").environ.get("PROBE_MAX_ITERS", "60000")), warm_start=True)
    tc = time.time() - t
    s = m.stats()
    bw = 8.0 * m.info.x_entries * s["x_pass_lp_iters"] / max(1e-9, s["x_pass_ms"] * 1e-3) / 1e9
    print(f"   children warm: st={r['status'].tolist()} it={r['iters'].tolist()} {tc:.2f}s "
          f"x_pass {s['x_pass_ms'] / max(1, s['x_pass_sampled']):.4f} ms/launch ~{bw:.0f} GB/s", flush=True)
    m.reset_stats()
    t = time.time()
    r = m.solve(np.arange(B), lb, ub, tol=1e-6, max_iters=int(__import__("os").environ.get("PROBE_MAX_ITERS", "60000")), warm_start=False)
    tc = time.time() - t
    s = m.stats()
    bw = 8.0 * m.info.x_entries * s["x_pass_lp_iters"] / max(1e-9, s["x_pass_ms"] * 1e-3) / 1e9
    print(f"   children cold: st={r['status'].tolist()} it={r['iters'].tolist()} {tc:.2f}s "
          f"x_pass {s['x_pass_ms'] / max(1, s['x_pass_sampled']):.4f} ms/launch ~{bw:.0f} GB/s", flush=True)
    m.close()
