#!/bin/bash
# round 2, call U: step-2 convergence probe (which side of the certificate lags)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 500 python -u tools/step2_probe.py syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization:1 syn_6x4_s1_r0.3_NeptuneMinDelay:1 payload:1 > $O/probe.log 2>&1
rc=$?; grep -v "amdgpu\|Initializ" $O/probe.log | tail -80; exit $rc
