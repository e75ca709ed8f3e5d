#!/bin/bash
# GPU box: parity suite, smoke, default bench and a longer (24-step) bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu27.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu27.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke27.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke27.log; [ $rc -eq 0 ] || exit $rc
for st in 24; do
  timeout -k 10 300 python -u bench.py --cpu-budget 0 --steps $st > gpurun_out/b27_s$st.json 2> gpurun_out/b27_s$st.log
  rc=$?; echo "bench steps $st rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/b27_s$st.json'));print(d['value'],d['ms_per_step'],d['lp'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'])"
done
