#!/bin/bash
# The GPU-box measurement recipes, parameterised (replaces the one-off round-2 call scripts; the index
# of what each past call measured is tools/gpu/README.md).  Run from this container as
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash tools/gpu/run.sh <out-name> <recipe> [<recipe> ...]
# Outputs go to gpurun_out/<out-name>/.  Every GPU step runs under its own time limit; the first failing
# step ends the call (no retries, nothing after a fault).  Recipes:
#   tests          python -m pytest tests -m gpu (all GPU tests, -x, per-test timeout)
#   tests:<files>  the GPU tests of the given comma-separated test files only
#   smoke          __graft_entry__.smoke()
#   bench          python bench.py (defaults: CPU baseline + product B&B sections included)
#   bench:<args>   python bench.py <args, comma-separated> (e.g. bench:--seed,1,--cpu-budget,0) -> bench_args<k>.json
#   env:<VAR>=<v>  export a variable for the following steps (e.g. env:NEPTUNE_LP_LIB=lib/variants/...); unenv:<VAR>
#   profile        rocprofv3 --kernel-trace --stats over the bench's timed replay -> kernel_stats_by_slots.csv
#   traffic        separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/traffic.py -> traffic.json
#   sq             SQ wave / wait / VALU counters of the steady x_pass -> sq.json
#   sq2            SQ LDS wait / bank-conflict / VMEM-read cycle counters of the steady x_pass -> sq2.json
#   probe:<args>   tools/probes/step2_probe.py <args, comma-separated>
#   kprof:<name>,<args>  rocprofv3 --kernel-trace --stats over a dev probe -> kprof_<name>.csv
#   py:<name>,<args>  a dev probe: python tools/probe.py <name> <args> (tools/probes/<name>.py), or a tools/*.py
#                  script (py:record_bnb_trace.py,...)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p "$O"
nb=0
npy=0
step() {   # step <name> <seconds> <command...>: run, log, stop the call on failure
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v "amdgpu\|Initializ" "$O/$name.log" | tail -25
  [ $rc -eq 0 ] || exit $rc
}
for r in "$@"; do
  case $r in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    tests:*) a=${r#tests:}; step pytest_sel 900 python -u -m pytest ${a//,/ } -m gpu -v -s --timeout 300 --timeout-method thread ;;
    smoke) step smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python -u bench.py ; grep "^{" "$O/bench.log" | tail -1 > "$O/bench.json" ;;
    bench:*) a=${r#bench:}; nb=$((nb + 1)); step bench_args$nb 600 python -u bench.py ${a//,/ }
      grep "^{" "$O/bench_args$nb.log" | tail -1 > "$O/bench_args$nb.json" ;;
    env:*) export "${r#env:}"; echo "== export ${r#env:}" ;;
    unenv:*) unset "${r#unenv:}"; echo "== unset ${r#unenv:}" ;;
    profile)
      step profile 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run -- python3 bench.py --steps 8 --cpu-budget 0 --bnb-seconds 0 --alibaba-seconds 0 --native-steps 0 --children-steps 0
      python3 tools/prof_summary.py /tmp/prof > "$O/kernel_stats_by_slots.csv"; cp /tmp/prof/*/*stats.csv "$O/" 2>/dev/null
      head -12 "$O/kernel_stats_by_slots.csv" | cut -c1-160 ;;
    traffic)
      # (ROC_AQL_QUEUE_SIZE: the default 16384-packet HSA queue crashes rocprofiler-sdk's --pmc queue intercept,
      # which reads a packet header one past the ring's end; DESIGN.md §6 "PMC pass crash")
      export ROC_AQL_QUEUE_SIZE=65536
      step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o run -- python3 tools/traffic.py run
      step pmc_write 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o run -- python3 tools/traffic.py run
      python3 tools/traffic.py summarize /tmp/pmc_fetch /tmp/pmc_write > "$O/traffic.json"; cat "$O/traffic.json" ;;
    sq)
      export ROC_AQL_QUEUE_SIZE=65536
      # (x_pass dispatches only, cold nodes — no 114k-iteration root solve: round 5's two passes outlived their limit
      # while rocprofv3 wrote a dispatch database of ~178k kernels)
      step pmc_sq 240 rocprofv3 --kernel-include-regex x_pass --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d /tmp/pmc_sq -o run -- python3 tools/traffic.py run cold
      python3 tools/traffic.py sq /tmp/pmc_sq > "$O/sq.json"; cat "$O/sq.json" ;;
    kprof:*) a=${r#kprof:}; n=${a%%,*}
      step "kprof_$n" 600 rocprofv3 --kernel-trace --stats -d /tmp/kprof_$n -o run -- python3 tools/probe.py ${a//,/ }
      cp /tmp/kprof_$n/*/*stats.csv "$O/" 2>/dev/null; python3 tools/prof_summary.py /tmp/kprof_$n > "$O/kprof_$n.csv"
      head -12 "$O/kprof_$n.csv" | cut -c1-160 ;;
    sq2)
      export ROC_AQL_QUEUE_SIZE=65536
      # LDS waits beside the memory waits of the steady x_pass (round 6: is the row loop waiting on LDS?)
      step pmc_sq2 240 rocprofv3 --kernel-include-regex x_pass --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD -d /tmp/pmc_sq2 -o run -- python3 tools/traffic.py run cold
      python3 tools/traffic.py sq /tmp/pmc_sq2 > "$O/sq2.json"; cat "$O/sq2.json" ;;
    probe:*) a=${r#probe:}; step probe 600 python -u tools/probe.py step2_probe ${a//,/ } ;;
    py:*) a=${r#py:}; n=${a%%,*}; n=${n%.py}; npy=$((npy + 1))
      if [ -f "tools/probes/$n.py" ]; then step "py${npy}_$n" 600 python -u tools/probe.py ${a//,/ }
      else step "py${npy}_$n" 600 python -u tools/${a//,/ }; fi ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
done
