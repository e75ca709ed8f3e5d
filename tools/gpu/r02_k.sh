#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02k; mkdir -p $O
for c in "testpy NeptuneWithEFTTCMinDelayAndUtilization" "syn_4x3_s0_r0.5_NeptuneMinDelayAndUtilization NeptuneWithEFTTCMinDelayAndUtilization"; do
  timeout -k 10 200 python -u tools/flow_probe.py $c >> $O/flow_probe.log 2>&1
  rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/flow_probe.log; exit $rc; }
done
grep -v "amdgpu\|Initializing" $O/flow_probe.log | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_gpu_bnb.py -q --timeout 200 --timeout-method thread -rf -s > $O/pytest_bnb.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed|'status'" $O/pytest_bnb.log | cut -c1-400 | tail -20
