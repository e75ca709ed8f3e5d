#!/bin/bash
# round 2, call AA: node-relocation local search on step-2 incumbents: Alibaba flows + B&B GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02aa; mkdir -p $O
timeout -k 10 600 python -u tools/alibaba_flow.py --step-seconds 45 --out $O/alibaba_flows.json > $O/alibaba.log 2>&1
rc=$?; echo "alibaba rc=$rc"; grep -v "amdgpu\|Initializ" $O/alibaba.log | cut -c1-300 | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bnb.py -x -v --timeout 180 --timeout-method thread > $O/pytest_bnb.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" $O/pytest_bnb.log | tail -8; exit $rc
