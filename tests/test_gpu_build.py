"""The model build from PyTorch-ROCm tensors (nep_model_desc.device_inputs, API 9) with the step size computed on
the device (nep_build.hip power iteration; DESIGN.md §6 "Device build"): the same eta = 0.95 / ||K̃||_2 as the host
build's power iteration (nep_debug_build, host arrays) on the same model — step 1, the facility relaxation and the
reduced step-2 block — to fp rounding (the device reads D / core_per_req in fp32), and the same scaling.  At
512x256 the build takes a fraction of the host power iteration's seconds."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [(64, 32, "MinDelayAndUtilization", 1, 0), (64, 32, "MinDelayAndUtilization", 1, 1),
         (64, 32, "MinUtilization", 3, 0), (64, 32, "MinDelay", 2, 0), (256, 128, "MinDelayAndUtilization", 1, 0)]


@pytest.mark.parametrize("n,f,variant,step,relax", CASES)
def test_device_build_step_size_equals_host(n, f, variant, step, relax):
    from core.engine.lp import LPModel, debug_build
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    data = data_to_solver_input(synthetic_payload(n, f, seed=0), with_db=False)
    kw = dict(alpha=0.5, relaxation=relax)
    if step != 1:
        kw.update(max_score=0.2, soften_step1_sol=1.3)
    host = debug_build(data, variant, step=step, **kw)
    m = LPModel(data, variant, step=step, max_batch=2, **kw)
    try:
        assert m.tensors["delay"].is_cuda and m.tensors["workload"].dtype.is_floating_point
        eta = m.info.step_size
        print(f"{n}x{f} {variant} step {step} relax {relax}: eta device {eta!r} host {host['eta']!r}")
        assert abs(eta / host["eta"] - 1.0) < 1e-6
        if step == 1:   # the device-built model solves: its root LP certifies (the step-2 models here have no
            # step-1 delay to soften — prev_network_delay 0 — so only their build is compared)
            r = m.solve([0], tol=1e-6, max_iters=200000)
            assert int(r["status"][0]) == 0, r
    finally:
        m.close()


def test_device_build_512x256_time():
    from core.engine.lp import LPModel
    from core.utils import data_to_solver_input
    from core.utils.synthetic import synthetic_payload
    data = data_to_solver_input(synthetic_payload(512, 256, seed=0), with_db=False)
    t0 = time.perf_counter()
    m = LPModel(data, "MinDelayAndUtilization", step=1, alpha=0.5, max_batch=2)
    t = time.perf_counter() - t0
    print(f"512x256 model build from device tensors: {t:.2f} s, eta {m.info.step_size!r}")
    m.close()
    assert t < 30.0


@pytest.mark.parametrize("name", ["syn64x32_MDU_s2delete", "syn64x32_MU_s2create"])
def test_device_build_step2_block(name):
    """The reduced step-2 block (D3/D4 folded into one row, dred) built from device tensors."""
    from core.engine.lp import LPModel, debug_build
    from scale_util import case_model_args, scale_cases
    data, variant, step, kw = case_model_args(scale_cases()[name])
    host = debug_build(data, variant, step=step, **kw)
    m = LPModel(data, variant, step=step, max_batch=1, **kw)
    try:
        assert abs(m.info.step_size / host["eta"] - 1.0) < 1e-6, (m.info.step_size, host["eta"])
    finally:
        m.close()


def test_one_hip_runtime_per_process():
    """The engine and PyTorch-ROCm share one HIP runtime (core/engine/lp.py load_library imports torch first):
    one libamdhip64 mapped, and a tensor torch wrote is read by the engine's build."""
    from core.engine.lp import load_library
    load_library()
    import torch
    torch.zeros(1, device="cuda")
    with open("/proc/self/maps") as fh:
        libs = {ln.split()[-1] for ln in fh if "libamdhip64" in ln}
    print("HIP runtime:", libs)
    assert len(libs) == 1, libs
