#!/bin/bash
# Round 4: the whole -m gpu suite
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_full}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s -rA --durations=30 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|XFAIL|ERROR|passed|failed" "$O/pytest_gpu.log" | grep -v "^tests.*PASSED$" | tail -40; exit $rc
