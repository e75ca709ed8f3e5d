#!/bin/bash
# GPU box: bench with the node-LP retry policy (defaults), retry after 512, retry off.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "" "--retry-after 512" "--retry-after 0"; do
  n=$(echo "x$v" | tr -d ' -')
  timeout -k 10 200 python -u bench.py --cpu-budget 0 $v > gpurun_out/b18_$n.json 2> gpurun_out/b18_$n.log
  rc=$?; echo "[$v] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/b18_$n.json'));print(d['value'],d['lp']['certified'],d['lp']['iterations'],d['lp']['iters_p50_p90_max'],d['roofline']['avg_launch_ms'])"
done
