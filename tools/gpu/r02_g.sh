#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 300 python -u tools/cert_probe.py sim0_NeptuneMinDelay:1 sim3_NeptuneMinUtilization:1 syn_8x4_s2_r0.1_NeptuneMinUtilization:0 > $O/cert_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu $O/cert_probe.log | cut -c1-250 | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_stream.py tests/test_gpu_params.py -q --timeout 300 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -40
exit $rc
