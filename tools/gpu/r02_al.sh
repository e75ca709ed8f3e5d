#!/bin/bash
# round 2, call AL: the two MinUtilization scale cases that failed under the warm primal-weight cap
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 600 python -u -m pytest "tests/test_gpu_scale.py::test_scale_parity[alibaba_MinUtilization_s1]" "tests/test_gpu_scale.py::test_scale_parity[syn64x32_MinUtilization_s1]" -q --timeout 300 --timeout-method thread -rf -s > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -v "amdgpu\|Initializ" $O/pytest.log | grep -E "Error|assert|iterations|FAILED|passed|failed" | cut -c1-300 | tail -20
NEP_X=1 timeout -k 10 600 python -u -c "
import sys; sys.path[:0]=['neptune-mip_amd','tests','.']
import test_gpu_scale as t, numpy as np
for cap in (0.0, -1.0, 16.0):
    for name in ('alibaba_MinUtilization_s1','syn64x32_MinUtilization_s1'):
        c=t.CASES[name]
        from core.engine.lp import LPModel
        from scale_util import case_model_args, node_bounds
        data, variant, step, kw = case_model_args(c)
        B=len(c['nodes']); m=LPModel(data, variant, step=step, max_batch=B+1, **kw)
        rr=m.solve([B], tol=t.SOLVE_TOL, max_iters=400000)
        lb,ub=node_bounds(c, m.n_int)
        for b in range(B): m.copy_state(B,b)
        res=m.solve(np.arange(B), lb, ub, tol=t.SOLVE_TOL, max_iters=200000, warm_start=True, warm_omega_cap=cap)
        print(cap, name, 'root', rr['status'][0], rr['iters'][0], 'nodes', res['status'].tolist(), res['iters'].tolist(), flush=True)
        m.close()
" > $O/caps.log 2>&1
rc=$?; echo "caps rc=$rc"; grep -v "amdgpu\|Initializ" $O/caps.log | tail -8
