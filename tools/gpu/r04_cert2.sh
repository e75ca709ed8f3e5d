#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_cert2}; mkdir -p "$O"
for it in 200000 400000; do
ITERS=$it timeout -k 10 200 python -u tools/step2_cert_probe.py syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization 1 3 > "$O/syn64_$it.log" 2>&1
rc=$?; echo "syn64 $it rc=$rc"; grep -v "amdgpu\|Initializ" "$O/syn64_$it.log" | tail -12
[ $rc -eq 0 ] || exit $rc
done
