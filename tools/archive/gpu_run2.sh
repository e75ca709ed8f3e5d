#!/bin/bash
# probe: convergence + bandwidth at growing sizes (no tests)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/probe_scale.py 64x32 128x64 256x128 512x256 > gpurun_out/probe2.log 2>&1
echo "probe rc=$?"
