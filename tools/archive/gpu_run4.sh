#!/bin/bash
# GPU box: parity tests, then the scale probe (root + warm/cold children at growing sizes).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu4.log 2>&1
rc=$?; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
PROBE_MAX_ITERS=100000 timeout -k 10 420 python -u tools/probe_scale.py 64x32 256x128 512x256 > gpurun_out/probe4.log 2>&1
rc=$?; echo "probe rc=$rc"
exit $rc
