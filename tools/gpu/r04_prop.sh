#!/bin/bash
# Round 4: step-2 bound propagation (D1/D2 -> c) in the presolve: the GPU parity suites of the LP
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_prop}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/step2_cert_probe.py payload 1 1 > "$O/payload.log" 2>&1
rc=$?; echo "payload rc=$rc"; grep -v "amdgpu\|Initializ" "$O/payload.log" | head -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_solvers.py tests/test_gpu_stream.py tests/test_gpu_bnb.py -m gpu -v -s -rA --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed|UNCERTIFIED" "$O/pytest.log" | tail -14; exit $rc
