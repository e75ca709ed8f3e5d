#!/bin/bash
# GPU box: drained-stream bench at warm-start primal-weight floors 2 and 4 (node-LP limit 4096).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for fl in 2 4; do
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --warm-omega-floor $fl > gpurun_out/b10_f$fl.json 2> gpurun_out/b10_f$fl.log
  rc=$?; echo "floor $fl rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/b10_f$fl.json'));print(d['value'],d['lp'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'])"
done
