#!/bin/bash
# GPU box: bench at check_every 16 / 24 / 32.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ce in ${CES:-16 24 32}; do
  timeout -k 10 200 python -u bench.py --cpu-budget 0 --check-every $ce > gpurun_out/b17_ce$ce.json 2> gpurun_out/b17_ce$ce.log
  rc=$?; echo "ce $ce rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/b17_ce$ce.json'));print(d['value'],d['lp']['certified'],d['lp']['iterations'],d['lp']['iters_p50_p90_max'],d['roofline']['avg_launch_ms'])"
done
