#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_cert}; mkdir -p "$O"
timeout -k 10 120 python -u tools/step2_cert_probe.py payload 1 1 > "$O/payload.log" 2>&1
rc=$?; echo "payload rc=$rc"; grep -v "amdgpu\|Initializ" "$O/payload.log" | tail -14
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/step2_cert_probe.py syn_4x3_s0_r0.5_NeptuneMinUtilization 1 3 > "$O/syn43.log" 2>&1
rc=$?; echo "syn43 rc=$rc"; grep -v "amdgpu\|Initializ" "$O/syn43.log" | tail -14; exit $rc
