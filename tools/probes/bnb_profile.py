#!/usr/bin/env python3
"""Dev probe (GPU box): the product step-1 search (NeptuneStepBase.branch_and_bound, two models) under
cProfile, time-limited — where the host's share of the B&B wall time goes (round-4 VERDICT item 9).

  python3 tools/bnb_profile.py 64x32:10 256x128:20
"""
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]


def run(N, F, secs):
    from core.engine.lp import LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    p = synthetic_payload(N, F, seed=0)
    data = data_to_solver_input(p, with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6, lp_max_iters=4096)
    st1.load_data(data)
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    bm = st1.bound_model(data, 33)
    bnb = st1.branch_and_bound(m, bm, time_limit=secs, root_max_iters=400000)
    pr = cProfile.Profile()
    t0 = time.time()
    pr.enable()
    res = bnb.solve()
    pr.disable()
    wall = time.time() - t0
    m.close()
    bm.close()
    d = res.as_dict()
    print(f"== {N}x{F} {secs}s: {res.status} inc {res.objective} bound {res.bound} nodes {res.nodes} lps {res.lps} "
          f"wall {wall:.1f}s timing {d['timing']}", flush=True)
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(28)
        print(s.getvalue(), flush=True)


def main():
    for arg in sys.argv[1:]:
        size, secs = arg.split(":")
        N, F = (int(t) for t in size.split("x"))
        run(N, F, float(secs))


if __name__ == "__main__":
    main()
