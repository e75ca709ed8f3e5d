#!/bin/bash
# Round 4: the facility relaxation (NEP_RELAX_FACILITY): GPU parity test, root/children probe, then the
# repaired-dual restart probe of the step-2 LPs (tools/gpu/r04_swap.sh)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_fac}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fac.py -m gpu -v -s --timeout 300 --timeout-method thread > "$O/pytest_fac.log" 2>&1
rc=$?; echo "pytest_fac rc=$rc"; grep -v "amdgpu\|Initializ" "$O/pytest_fac.log" | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u tools/fac_probe.py 64x32 256x128 512x256 > "$O/fac_probe.log" 2>&1
rc=$?; echo "fac_probe rc=$rc"; tail -20 "$O/fac_probe.log"
[ $rc -eq 0 ] || exit $rc

