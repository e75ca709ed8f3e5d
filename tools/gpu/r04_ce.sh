#!/bin/bash
# Round 4: certificate interval on the replay stream (check_every 12 / 24 / 48)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_ce}; mkdir -p "$O"
for ce in 12 24 48; do
  timeout -k 10 300 python -u bench.py --steps 6 --check-every $ce --native-steps 0 --children-steps 12 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_ce$ce.json" 2> "$O/bench_ce$ce.err"
  rc=$?; echo "bench ce=$ce rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_ce$ce.json'));print(d['value'], d['lp']['certified'], d['lp']['completed'], d['lp']['mean_iters'], d['roofline']['frac'], d['children_stream']['value'])"
  [ $rc -eq 0 ] || exit $rc
done
for kn in '{"root_check_every": 64}' '{"root_check_every": 12}'; do
  tag=$(echo $kn | tr -dc 0-9)
  MODES=two KNOBS="$kn" timeout -k 10 200 python -u tools/bnb_fac_probe.py 256x128:20 512x256:20 > "$O/bnb_rce$tag.log" 2>&1
  rc=$?; echo "bnb [$kn] rc=$rc"; grep "two\|mix" "$O/bnb_rce$tag.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --steps 6 --warm-ancestors --native-steps 0 --children-steps 0 --bnb-seconds 0 --cpu-budget 0 > "$O/bench_anc.json" 2> "$O/bench_anc.err"
rc=$?; echo "bench ancestors rc=$rc"; python3 -c "import json;d=json.load(open('$O/bench_anc.json'));print(d['value'], d['lp']['certified'], d['lp']['completed'], d['lp']['mean_iters'], d['lp']['warm_from_parent_rank0'])"
