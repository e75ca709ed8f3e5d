#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 400 python -u tools/cert_probe.py > $O/cert_probe.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu $O/cert_probe.log | cut -c1-330 | head -60
exit $rc
