#!/bin/bash
# round 2, call V: CPU-row repair at certificate iterations: bench (tail), then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02v; mkdir -p $O
timeout -k 10 400 python -u bench.py --cpu-budget 0 --bnb-seconds 20 > $O/bench.json 2> $O/bench.log
rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 $O/bench.log; exit $rc; }
python -c "import json;d=json.load(open('$O/bench.json'));l=d['lp'];print('bench', round(d['value'],1), l['certified'], l['completed'], round(l['mean_iters'],1), l['iters_p50_p90_max'], round(d['roofline']['avg_launch_ms'],3), round(d['roofline']['frac'],3), d['ms_per_step'], 'root', l['root_iters']); b=d.get('bnb',{}); print('bnb', {k: b.get(k) for k in ('status','nodes','lps','certified_lps','incumbent','bound')})"
timeout -k 10 1300 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; grep -c UNCERTIFIED $O/pytest_gpu.log; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -8; exit $rc
