#!/bin/bash
# round 3, call A: which side of the step-2 certificate lags (pobj vs HiGHS, best bound vs HiGHS)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03a; mkdir -p $O
BUDGETS=2000,20000,200000 timeout -k 10 420 python -u tools/step2_probe.py syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization:1 \
  syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization:1 syn_6x4_s1_r0.3_NeptuneMinDelay:1 payload:1 \
  scale:syn64x32_MDU_s2create scale:syn64x32_MDU_s2delete > $O/probe.log 2>&1
rc=$?; grep -v "amdgpu\|Initializ" $O/probe.log | tail -120; exit $rc
