#!/bin/bash
# round 3, call B: dual repair of the big-M row pairs — step-2 probe, LP / scale parity tests; B&B CPU repair
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03b; mkdir -p $O
BUDGETS=2000,20000,200000 timeout -k 10 300 python -u tools/step2_probe.py syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization:1 \
  syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization:1 syn_6x4_s1_r0.3_NeptuneMinDelay:1 payload:1 \
  scale:syn64x32_MDU_s2create scale:syn64x32_MDU_s2delete > $O/probe.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_bnb.py -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -v "amdgpu\|Initializ" $O/probe.log | tail -75; grep -E "UNCERTIFIED|passed|failed|FAILED|iterations|lp_status" $O/pytest.log | tail -60; exit $rc
