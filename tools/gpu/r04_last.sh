#!/bin/bash
# Round 4: the whole -m gpu suite and smoke() on the final head
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_last}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rA --durations=15 --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest_gpu.log" | grep -v "PASSED" | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke.log"; exit $rc
