#!/bin/bash
# GPU box: bench at 4 / 8 / 16 waves per x-pass workgroup (NEP_TILE_WAVES, dev knob).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for tw in 4 16 8; do
  NEP_TILE_WAVES=$tw timeout -k 10 200 python -u bench.py --cpu-budget 0 > gpurun_out/b12_tw$tw.json 2> gpurun_out/b12_tw$tw.log
  rc=$?; echo "tw $tw rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep "root LP" gpurun_out/b12_tw$tw.log
  python -c "import json;d=json.load(open('gpurun_out/b12_tw$tw.json'));print(d['value'],d['lp']['certified'],d['lp']['iterations'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'],d['roofline']['algorithmic_bytes_per_launch']/55.5e6)"
done
