#!/bin/bash
# round 2, call P: node LPs in flight per GPU (32 / 64 / 128, same 768 nodes), then the Alibaba flows
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02p; mkdir -p $O
for bs in "32 24" "64 12" "128 6"; do
  set -- $bs
  timeout -k 10 240 python -u bench.py --batch $1 --steps $2 --cpu-budget 0 --bnb-seconds 0 > $O/b_$1.json 2> $O/b_$1.log
  rc=$?; [ $rc -eq 0 ] || { echo "batch $1 rc=$rc"; tail -3 $O/b_$1.log; exit $rc; }
  python -c "import json;d=json.load(open('$O/b_$1.json'));l=d['lp'];print('batch $1', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3), d['ms_per_step'])"
done
timeout -k 10 900 python -u tools/alibaba_flow.py --step-seconds 45 --out $O/alibaba_flows.json > $O/alibaba.log 2>&1
rc=$?; echo "alibaba rc=$rc"; grep -v "amdgpu\|Initializ" $O/alibaba.log | cut -c1-300 | tail -20
