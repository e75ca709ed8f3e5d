#!/bin/bash
# Round 5: the 512x256 product B&B under the three ways the engine gets its instance and step size:
# PyTorch-ROCm tensors + device eta (default), tensors + host eta, host arrays on /opt/rocm's runtime
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_rt}; mkdir -p "$O"; S=${2:-60}
timeout -k 10 300 python -u tools/bnb_ab.py 512 256 $S > "$O/default.json" 2> "$O/default.err" || exit $?
tail -c 600 "$O/default.json"; echo
NEP_HOST_POWER=1 timeout -k 10 300 python -u tools/bnb_ab.py 512 256 $S > "$O/hostpower.json" 2> "$O/hostpower.err" || exit $?
tail -c 600 "$O/hostpower.json"; echo
NEP_HOST_INPUTS=1 timeout -k 10 300 python -u tools/bnb_ab.py 512 256 $S > "$O/hostinputs.json" 2> "$O/hostinputs.err" || exit $?
tail -c 600 "$O/hostinputs.json"; echo
