#!/bin/bash
# round 2, call X: Alibaba MDU flow with the disruption-block bound, verbose (incumbent timing), then
# the same with the step-2 bound disabled (NEP_DBLOCK=0) for comparison
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02x; mkdir -p $O
cat > $O/run.py <<'PY'
import json, os, sys, time
sys.path[:0] = ["neptune-mip_amd", ".", "tests"]
import core.solvers as S
from core.utils import data_to_solver_input
p = json.load(open("tests/golden/inputs/alibaba_NeptuneMinDelayAndUtilization.json"))
args = dict(p["solver"].get("args", {})); args.update(time_limit=45.0, verbose=True)
s = S.SOLVERS["NeptuneMinDelayAndUtilization"](**args)
s.load_data(data_to_solver_input(p, workload_coeff=1, with_db=False))
t = time.time(); s.solve(); print("score", s.score(), time.time() - t, flush=True)
print("create", s.step2_create.result.as_dict())
PY
timeout -k 10 200 python -u $O/run.py > $O/mdu.log 2>&1
rc=$?; grep -v "amdgpu\|Initializ" $O/mdu.log | cut -c1-250 | tail -25; exit $rc
