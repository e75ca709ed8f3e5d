#!/bin/bash
# round 2, call AT: polishing extended to step 2 — full GPU suite (uncertified step-2 LPs counted), Alibaba flows
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02at; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rf -s > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -20; echo "uncertified: $(grep -c UNCERTIFIED $O/pytest_gpu.log)"
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
timeout -k 10 600 python -u tools/alibaba_flow.py --step-seconds 45 --out $O/alibaba_flows.json > $O/alibaba.log 2>&1
rc=$?; echo "alibaba rc=$rc"; grep -v "amdgpu\|Initializ" $O/alibaba.log | cut -c1-300 | tail -8
