#!/bin/bash
# round 2, call S: Alibaba flows with step-2 primal starts, the delete-mode opening-count prune and
# LP-c-first rounding, minimal-opening leaves and the step-2 integral bound; then the product B&B / EF-TTC GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 600 python -u tools/alibaba_flow.py --step-seconds 45 --out $O/alibaba_flows.json > $O/alibaba.log 2>&1
rc=$?; echo "alibaba rc=$rc"; grep -v "amdgpu\|Initializ" $O/alibaba.log | cut -c1-300 | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_bnb.py -x -v --timeout 180 --timeout-method thread > $O/pytest_bnb.log 2>&1
rc=$?; tail -5 $O/pytest_bnb.log; exit $rc
