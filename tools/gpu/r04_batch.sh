#!/bin/bash
# Round 4 batch (one GPU call): parity tests of the step-2 goldens with the widened pooled shift, the facility
# relaxation and sharded-B&B GPU tests, the primal-leaf probe, and the 512x256 B&B trace for bench.py's replay
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_batch}; mkdir -p "$O"
run() {   # run <name> <seconds> <cmd...>: rc 0/1 (test failures) continue, anything else stops the call
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v "amdgpu\|Initializ" "$O/$name.log" | grep -E "PASS|FAIL|XFAIL|passed|failed|Error|rc=|: |LP " | tail -${TAILN:-25}
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run lp_goldens 400 python -u -m pytest tests/test_gpu_lp.py -m gpu -v -s --timeout 300 --timeout-method thread -k "payload or syn_4x3_s0_r0.5_NeptuneMinUtilization or syn_6x4_s1_r0.3_NeptuneMinDelayAndUtilization"
run fac_dist 600 python -u -m pytest tests/test_gpu_fac.py tests/test_gpu_bnb_dist.py -m gpu -v -s --timeout 300 --timeout-method thread
run leaf 500 python -u tools/leaf_probe.py 64x32 128x64 256x128
run trace 200 python -u tools/record_bnb_trace.py 512 256 60 "$O"
