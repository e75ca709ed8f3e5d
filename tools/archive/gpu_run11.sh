#!/bin/bash
# GPU box: parity suite, then the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu11.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu11.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-budget 0 > gpurun_out/b11.json 2> gpurun_out/b11.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/b11.json'));print(d['value'],d['ms_per_step'],d['lp'],d['roofline'])"
