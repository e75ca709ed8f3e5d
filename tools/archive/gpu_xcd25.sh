#!/bin/bash
# GPU box: bench + FETCH/WRITE_SIZE passes with the XCD-aware x-pass workgroup order.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r25
timeout -k 10 300 python -u bench.py --cpu-budget 0 > gpurun_out/r25/bench.json 2> gpurun_out/r25/bench.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json;d=json.load(open('gpurun_out/r25/bench.json'));print(d['value'],d['lp']['certified'],d['lp']['iterations'],d['roofline']['achieved'],d['roofline']['avg_launch_ms'])"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/r25/pmc_fetch -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/r25/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/r25/pmc_write -o run -- python3 $R/tools/traffic.py run > $R/gpurun_out/r25/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 tools/traffic.py summarize gpurun_out/r25/pmc_fetch gpurun_out/r25/pmc_write > gpurun_out/r25/traffic.json && cat gpurun_out/r25/traffic.json
