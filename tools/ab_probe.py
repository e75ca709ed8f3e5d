#!/usr/bin/env python3
"""Dev probe (GPU box): root + first-check diagnostics of warm children, to A/B two engine builds
(select the build with NEPTUNE_LP_LIB).  Prints the root's iterations / objective / diagnostics and,
for the bench's first children, the status and certificate terms after one block."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:])
    import torch
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    torch.cuda.set_device(0)
    p = synthetic_payload(a.nodes, a.functions, seed=a.seed)
    d = data_to_solver_input(p, with_db=False)
    m = LPModel(d, "MinDelayAndUtilization", step=1, alpha=p["solver"]["args"]["alpha"], max_batch=9)
    root = 8
    for cut in (64, 128, 1024):
        r = m.solve([root], tol=a.tol, max_iters=cut, check_every=a.root_check_every)
        dg = m.diag(root)
        print(f"root cut {cut}: st {r['status'][0]} it {r['iters'][0]} obj {r['obj'][0]:.10g} pobj {dg['pobj']:.10g} "
              f"pres {dg['pres']:.3g} gap {dg['gap']:.3g} omega {dg['omega']:.4g} ksr {dg['k_since_restart']:.0f}",
              flush=True)
    r = m.solve([root], tol=a.tol, max_iters=a.root_max_iters, check_every=a.root_check_every)
    dg = m.diag(root)
    print(f"root: st {r['status'][0]} it {r['iters'][0]} obj {r['obj'][0]:.10g} pobj {dg['pobj']:.10g} "
          f"pres {dg['pres']:.3g} gap {dg['gap']:.3g} omega {dg['omega']:.4g}", flush=True)
    lbs, ubs = [], []
    for k in range(8):
        lb, ub = bench.node_bounds(m.n_int, a.functions, a.nodes, 1, a.fix, (a.seed * 1000003) * 7919 + k)
        lbs.append(lb[0])
        ubs.append(ub[0])
        m.copy_state(root, k)
    for it in (1, a.check_every, 4 * a.check_every):
        for k in range(8):
            m.copy_state(root, k)
        rr = m.solve(np.arange(8), np.array(lbs), np.array(ubs), tol=a.tol, max_iters=it,
                     check_every=a.check_every, warm_start=True)
        for k in range(8):
            dg = m.diag(k)
            print(f"  child {k} max_it {it}: st {rr['status'][k]} it {rr['iters'][k]} obj {rr['obj'][k]:.10g} "
                  f"pobj {dg['pobj']:.10g} pres {dg['pres']:.3g} gap {dg['gap']:.3g} omega {dg['omega']:.4g}",
                  flush=True)
    m.close()


if __name__ == "__main__":
    main()
