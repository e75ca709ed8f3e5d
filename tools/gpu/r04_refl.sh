#!/bin/bash
# Round 4: the whole -m gpu suite on the NEP_INLINE_REFLECT build (lib/variants/libneptune_lp_refl.so), then
# the bench's replay + children streams on both builds
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_refl}; mkdir -p "$O"
export TMPDIR=/tmp
NEPTUNE_LP_LIB=$PWD/neptune-mip_amd/lib/variants/libneptune_lp_refl.so timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread > "$O/pytest_refl.log" 2>&1
rc=$?; echo "pytest refl rc=$rc"; grep -E "FAILED|XFAIL|XPASS|ERROR|passed|failed" "$O/pytest_refl.log" | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in default refl; do
  if [ $lib = refl ]; then export NEPTUNE_LP_LIB=$PWD/neptune-mip_amd/lib/variants/libneptune_lp_refl.so; else unset NEPTUNE_LP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 8 --native-steps 0 --children-steps 24 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_$lib.json" 2> "$O/bench_$lib.err"
  rc=$?; echo "bench $lib rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_$lib.json'));print(d['value'], d['lp']['iters_p50_p90_max'], d['lp']['warm_from_parent_rank0'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['children_stream']['value'])"
  [ $rc -eq 0 ] || exit $rc
done
