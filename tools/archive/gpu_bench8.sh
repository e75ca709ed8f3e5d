#!/bin/bash
# GPU box: bench variants after the warm-start primal-weight floor (batch, check cadence).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "--batch 16" "--batch 32" "--batch 16 --check-every 32" "--batch 32 --check-every 32"; do
  n=$(echo $v | tr -d ' -')
  timeout -k 10 150 python -u bench.py --warmup 3 --steps 6 --cpu-budget 0 $v > gpurun_out/b8_$n.json 2> gpurun_out/b8_$n.log
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/b8_$n.json'));print(d['value'],d['lp'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'])"
done
