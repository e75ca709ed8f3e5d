#!/bin/bash
# Round 4: record the product B&B's node trace at 512x256 (the replay fixture), the facility GPU parity test,
# then bench.py on the fresh trace (no CPU baseline)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_bench}; mkdir -p "$O/trace"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/record_bnb_trace.py 512 256 ${TRACE_SECS:-60} "$O/trace" > "$O/record.log" 2>&1
rc=$?; echo "record rc=$rc"; grep -v "amdgpu\|Initializ" "$O/record.log" | tail -3
[ $rc -eq 0 ] || exit $rc
cp "$O/trace/bnb_trace_512x256_s0.json" tests/golden/
timeout -k 10 400 python -u -m pytest tests/test_gpu_fac.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest_fac.log" 2>&1
rc=$?; echo "pytest_fac rc=$rc"; grep "passed\|failed\|Error" "$O/pytest_fac.log" | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u bench.py --cpu-budget 0 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -5 "$O/bench.err"; cat "$O/bench.json"; exit $rc
