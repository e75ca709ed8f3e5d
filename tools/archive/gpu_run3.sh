#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PROBE_MAX_ITERS=100000 timeout -k 10 400 python -u tools/probe_scale.py 64x32 128x64 256x128 512x256 > gpurun_out/probe3.log 2>&1
rc=$?; echo "probe rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu3.log 2>&1
echo "pytest rc=$?"
