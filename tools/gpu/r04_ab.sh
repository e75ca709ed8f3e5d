#!/bin/bash
# Round 4 A/B: leaf routing warm starts in the two-model B&B; certificate x_pass at 3 waves/SIMD (cw3 build)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_ab}; mkdir -p "$O"
for kn in '{"leaf_routing_warm": true}' '{"leaf_routing_warm": false}'; do
  tag=$(echo $kn | tr -dc a-z)
  MODES=two KNOBS="$kn" timeout -k 10 200 python -u tools/bnb_fac_probe.py 256x128:20 512x256:20 > "$O/bnb_$tag.log" 2>&1
  rc=$?; echo "bnb [$kn] rc=$rc"; grep "two\|mix" "$O/bnb_$tag.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
for lib in default cw3; do
  if [ $lib = cw3 ]; then export NEPTUNE_LP_LIB=$PWD/neptune-mip_amd/lib/variants/libneptune_lp_cw3.so; else unset NEPTUNE_LP_LIB; fi
  timeout -k 10 300 python -u bench.py --steps 6 --native-steps 0 --children-steps 24 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_$lib.json" 2> "$O/bench_$lib.err"
  rc=$?; echo "bench $lib rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_$lib.json'));print(d['value'], d['lp']['root_iters'], d['lp']['root_seconds'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['children_stream']['value'])"
  [ $rc -eq 0 ] || exit $rc
done
