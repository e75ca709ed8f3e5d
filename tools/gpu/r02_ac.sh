#!/bin/bash
# round 2, call AC: sparse Halpern anchor — routing-row sparsity probe, LP parity tests, bench, PMC traffic
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 300 python -u tools/sparsity_probe.py > $O/sparsity.log 2>&1
rc=$?; echo "sparsity rc=$rc"; grep -v "amdgpu\|Initializ" $O/sparsity.log | cut -c1-400 | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_lp.py tests/test_gpu_scale.py tests/test_gpu_params.py tests/test_gpu_aux.py -q --timeout 300 --timeout-method thread -rf > $O/pytest_lp.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lp.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --cpu-budget 0 --bnb-seconds 0 > $O/bench.json 2> $O/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value'],1), d['lp'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 tools/traffic.py run > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 tools/traffic.py run > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic.py summarize $O/pmc_fetch $O/pmc_write > $O/traffic.json; cat $O/traffic.json
