#!/usr/bin/env python3
"""Dev probe (GPU box): the bench's cold root LP (512x256 step-1 MDU reference model, seed 0) under
restart / primal-weight settings — the round-4 VERDICT item on root latency.  Each setting is
"name" or "name:ENV=VAL;ENV=VAL" (read by nep_model_create); one model per setting.

  python3 tools/root_probe.py base "r85:NEP_RESTART=0.2,0.85,0.36" "sm3:NEP_OMEGA_SMOOTH=0.3"
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "neptune-mip_amd"), REPO]

KNOBS = ("NEP_RESTART", "NEP_OMEGA_SMOOTH", "NEP_POLISH")


def main():
    import torch
    torch.cuda.set_device(0)
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    N, F = int(os.environ.get("ROOT_N", 512)), int(os.environ.get("ROOT_F", 256))
    check = int(os.environ.get("ROOT_CHECK", 64))
    p = synthetic_payload(N, F, seed=int(os.environ.get("ROOT_SEED", 0)))
    data = data_to_solver_input(p, with_db=False)
    alpha = p["solver"]["args"]["alpha"]
    for arg in sys.argv[1:] or ["base"]:
        name, _, envs = arg.partition(":")
        for k in KNOBS:
            os.environ.pop(k, None)
        for kv in filter(None, envs.split(";")):
            k, _, v = kv.partition("=")
            os.environ[k] = v.replace("/", ",")   # ("/" for "," in values: tools/gpu/run.sh splits arguments on ",")
        m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=alpha, max_batch=2)
        t = time.perf_counter()
        r = m.solve([0], tol=1e-6, max_iters=int(os.environ.get("ROOT_MAX", 400000)), check_every=check)
        dt = time.perf_counter() - t
        d = m.diag(0)
        print(f"{name:10s} {envs:40s} status {int(r['status'][0])} obj {float(r['obj'][0]):.10g} "
              f"iters {int(r['iters'][0])} {dt:.2f}s | pobj {d['pobj']:.10g} best bound {d['best_lagr']:.10g} "
              f"primal residual {d['pres']:.3g} gap {d['gap']:.3g} omega {d['omega']:.3g}", flush=True)
        m.close()


if __name__ == "__main__":
    main()
