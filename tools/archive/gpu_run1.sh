#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u tools/probe_scale.py 64x32 256x128 512x256 > gpurun_out/probe.log 2>&1
echo "probe rc=$?"
