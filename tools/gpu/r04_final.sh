#!/bin/bash
# Round 4 closing measurement: bench.py (defaults), its rocprofv3 kernel-trace summary, the x_pass PMC traffic
# passes (FETCH_SIZE, WRITE_SIZE) on the replay workload, then bench.py again with the traffic file in place
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_final}; mkdir -p "$O"
export TMPDIR=/tmp
NEP_AUX_PRIORITY=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- python3 tools/traffic.py run > "$O/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
NEP_AUX_PRIORITY=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run -- python3 tools/traffic.py run > "$O/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic.py summarize "$O/pmc_fetch" "$O/pmc_write" > "$O/traffic.json" && cp "$O/traffic.json" profiles/traffic.json
rc=$?; echo "summarize rc=$rc"; cat "$O/traffic.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$O/bench.err"; cat "$O/bench.json"; exit $rc
