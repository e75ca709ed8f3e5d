"""The step-1 B&B at N x F for `seconds`, one JSON line of its result: an A/B probe for engine / runtime
settings taken from the environment (NEP_HOST_INPUTS, NEP_HOST_POWER, NEPTUNE_LP_LIB, BNB_WREF = the B&B's
warm_weight_ref).  BNB_MODE=single (default): tests/test_gpu_bnb.py::test_product_bnb_time_limited's one-model
search; BNB_MODE=product: the product's two-model search (NeptuneStepBase.branch_and_bound, as bench.py's bnb
section runs it).  Usage: python tools/bnb_ab.py N F seconds [seed]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neptune-mip_amd"))


def main():
    n, f, seconds = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    from core.engine.bnb import BranchAndBound
    from core.engine.lp import LPModel
    from core.solvers.neptune.neptune_step import NeptuneStep1CPUMinDelayAndUtilization
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    data = data_to_solver_input(synthetic_payload(n, f, seed=seed), with_db=False)
    st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False)
    st1.load_data(data)
    ub = st1.upper_bound()
    t0 = time.perf_counter()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=34)
    build = time.perf_counter() - t0
    bm = None
    wref = float(os.environ.get("BNB_WREF", "8"))
    try:
        if os.environ.get("BNB_MODE", "single") == "product":
            st1 = NeptuneStep1CPUMinDelayAndUtilization(alpha=0.5, verbose=False, batch=32, lp_tol=1e-6, lp_max_iters=4096)
            st1.load_data(data)
            st1.bound_park = int(os.environ.get("BNB_PARK", st1.bound_park))
            bm = st1.bound_model(data, 33)
            res = st1.branch_and_bound(m, bm, time_limit=seconds, root_max_iters=400000, warm_weight_ref=wref).solve()
        else:
            res = BranchAndBound(m, data.workload_matrix, data.function_memory_matrix, data.node_memory_matrix,
                                 batch=32, tol=5e-7 if n < 512 else 1e-6, time_limit=seconds,
                                 root_max_iters=200000 if n < 512 else 400000, upper_bound=ub * (1 + 1e-6) + 1e-6,
                                 repair=st1.routing_repair(m.layout()), warm_weight_ref=wref).solve()
    finally:
        m.close()
        if bm is not None:
            bm.close()
    d = res.as_dict()
    d["build_seconds"] = build
    d["eta"] = m.info.step_size
    d["env"] = {k: os.environ.get(k) for k in ("NEP_HOST_INPUTS", "NEP_HOST_POWER", "NEPTUNE_LP_LIB", "BNB_WREF",
                                                "BNB_MODE", "BNB_PARK")}
    with open("/proc/self/maps") as fh:
        d["hip_runtime"] = sorted({ln.split()[-1] for ln in fh if "libamdhip64" in ln})
    print(json.dumps(d, default=float))


if __name__ == "__main__":
    main()
