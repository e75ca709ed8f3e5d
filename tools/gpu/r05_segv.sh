#!/bin/bash
# Round 5: the round-4 SIGSEGV of the first rocprofv3 --pmc FETCH_SIZE pass (profiles/r04/final/
# pmc_fetch_segv_first_try.log), under its original conditions: root solve included, default (high) aux
# priority.  One pass; the call ends at its first failure.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_segv}; mkdir -p "$O"
export TMPDIR=/tmp
env ${NEP_ENV:-NEP_NONE=0} timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run -- python3 tools/traffic.py run > "$O/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; tail -40 "$O/pmc_fetch.log" | cut -c1-200; exit $rc
