#!/bin/bash
# round 2, call I: kernel-trace profile of the bench, PMC FETCH/WRITE passes, plain-PDHG A/B
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.log
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py $O/prof > $O/kernel_stats_by_slots.csv; head -12 $O/kernel_stats_by_slots.csv | cut -c1-160
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -- python3 tools/traffic.py run > $O/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -- python3 tools/traffic.py run > $O/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/traffic.py summarize $O/pmc_fetch $O/pmc_write > $O/traffic.json; cat $O/traffic.json
for v in default plain; do
  if [ $v = default ]; then lib=neptune-mip_amd/lib/libneptune_lp.so; else lib=neptune-mip_amd/lib/variants/libneptune_lp_$v.so; fi
  NEPTUNE_LP_LIB=$PWD/$lib timeout -k 10 240 python -u bench.py --steps 12 --cpu-budget 0 --bnb-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.log
  rc=$?; echo "bench $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['value'],1), d['lp']['certified'], d['lp']['completed'], round(d['lp']['mean_iters'],1), d['lp']['root_iters'], round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],3))"
done
