#!/usr/bin/env python3
"""Dev probe (GPU box): the certificate's primal side of one LP.  Solves a golden / scale case's root
(and nodes) cold to a budget, then saves the routing rows, the PDHG iterate's small variables and the
diagnostics to gpurun_out/<out>/primal_<case>.npz for an offline comparison with the HiGHS solution
(tools/primal_analyze.py, CPU).

  python3 tools/primal_probe.py <out-dir> scale:syn64x32_MDU_s2delete [budget]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402


def main():
    from core.engine.lp import LPModel
    from step2_probe import case
    out, arg = sys.argv[1], sys.argv[2]
    budget = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
    data, variant, step, kw, rootref, nodes, scale = case(arg)
    m = LPModel(data, variant, step=step, max_batch=1, **kw)
    res = m.solve([0], tol=5e-7, max_iters=budget, check_every=64)
    xb, rf, rs = m.rows(0)
    z, _ = m.solution(0, dense_x=False)
    dg = m.diag(0)
    from core.engine.lp import debug_build
    st = m.debug_state(0, debug_build(data, variant, step=step, **kw)["n_dual"])
    print(arg, "status", res["status"][0], "iters", res["iters"][0], "pobj", dg["pobj"], "bestL", dg["best_lagr"],
          "ref", rootref, "res", dg["pres"], flush=True)
    os.makedirs(out, exist_ok=True)
    np.savez(os.path.join(out, "primal_" + arg.replace(":", "_") + ".npz"), xb=xb, rf=rf, rs=rs, z=z,
             pobj=dg["pobj"], bestl=dg["best_lagr"], y=st["y"], ref=rootref, status=res["status"][0], iters=res["iters"][0])
    m.close()


if __name__ == "__main__":
    main()
