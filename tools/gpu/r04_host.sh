#!/bin/bash
# Round 4: host-path changes (one-copy submits, batched solution reads): the GPU tests that drive them, then
# the B&B host profile
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_host}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aux.py tests/test_gpu_stream.py tests/test_gpu_params.py tests/test_gpu_bnb.py tests/test_gpu_bnb_dist.py tests/test_gpu_bnb_parity.py tests/test_gpu_solvers.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$O/pytest.log" | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 150 python -u tools/bnb_profile.py 64x32:10 256x128:20 > "$O/profile.log" 2>&1
rc=$?; echo "profile rc=$rc"; grep "^==" "$O/profile.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --steps 4 --native-steps 0 --children-steps 4 --bnb-seconds 0 --cpu-budget 0 > "$O/prof_bench.json" 2> "$O/prof_bench.err"
rc=$?; echo "rocprof rc=$rc"; exit $rc
