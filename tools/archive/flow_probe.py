#!/usr/bin/env python3
"""Dev probe (GPU box): the NEPTUNE two-step flow on golden payloads with the B&B's node-LP
iteration limit PROBE_ITERS (comma list): wall time per step, B&B statistics, scores."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO, os.path.join(REPO, "tests")]


def main():
    import torch
    import core.solvers as S
    from core.utils import data_to_solver_input
    from golden_util import golden, payload
    torch.cuda.set_device(0)
    G = golden()
    for name in os.environ.get("PROBE_CASES", "payload,testpy,syn_4x3_s0_r0.5_NeptuneMinDelay").split(","):
        p = payload(name)
        ref = G[name]["response"]["score"]
        for its in [int(v) for v in os.environ.get("PROBE_ITERS", "100000,20000,5000").split(",")]:
            data = data_to_solver_input(p, workload_coeff=p.get("workload_coeff", 1), with_db=False)
            args = dict(p["solver"].get("args", {}))
            solver = S.SOLVERS[p["solver"]["type"]](lp_max_iters=its, **args)
            solver.load_data(data)
            t = time.perf_counter()
            solver.solve()
            dt = time.perf_counter() - t
            sc = solver.score()
            steps = [st.result.as_dict() for st in (solver.step1, solver.step2_delete, solver.step2_create)
                     if getattr(st, "result", None) is not None]
            print(f"{name} iters {its}: {dt:.2f}s score {sc} ref {ref}", flush=True)
            for d in steps:
                print("    ", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items()}, flush=True)


if __name__ == "__main__":
    main()
