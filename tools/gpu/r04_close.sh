#!/bin/bash
# Round 4 closing: the whole -m gpu suite, smoke(), the B&B host profile, then the default bench
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_close}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rA --durations=20 --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest_gpu.log" | grep -v "PASSED" | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -2 "$O/bench.err"; python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['lp']['certified'], d['lp']['completed'], d['roofline']['frac'], d['roofline']['traffic_over_algorithmic'], [ (b['workload'], b['rel_gap'], b['time_limit_s']) for b in d['bnb']])"; exit $rc
