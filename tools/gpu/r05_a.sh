#!/bin/bash
# Round 5: full -m gpu suite + smoke on the reduced step-2 block, then the replay bench with and without parked
# parent states (A/B; CPU baseline and the B&B / native / children sections skipped)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_a}; mkdir -p "$O"
export TMPDIR=/tmp
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?;
        echo "   rc=$rc"; tail -4 "$O/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()"
Q="--cpu-budget 0 --bnb-seconds 0 --native-steps 0 --children-steps 0 --steps 12"
run bench_park256 300 python -u bench.py $Q --park 256
run bench_park0 300 python -u bench.py $Q --park 0
