#!/bin/bash
# Round 4: artificial-restart threshold around the default on two seeds and 256x128 (tools/root_probe.py)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04_root2}; mkdir -p "$O"
export TMPDIR=/tmp
S="base art1:NEP_RESTART=0.2,0.9,0.1 art15:NEP_RESTART=0.2,0.9,0.15 art2:NEP_RESTART=0.2,0.9,0.2 art25:NEP_RESTART=0.2,0.9,0.25 art3:NEP_RESTART=0.2,0.9,0.3"
timeout -k 10 300 python -u tools/root_probe.py $S > "$O/root_s0.log" 2>&1
rc=$?; echo "s0 rc=$rc"; grep -v -e Warn -e amdgpu.ids "$O/root_s0.log"; [ $rc -eq 0 ] || exit $rc
ROOT_SEED=1 timeout -k 10 300 python -u tools/root_probe.py $S > "$O/root_s1.log" 2>&1
rc=$?; echo "s1 rc=$rc"; grep -v -e Warn -e amdgpu.ids "$O/root_s1.log"; [ $rc -eq 0 ] || exit $rc
ROOT_N=256 ROOT_F=128 timeout -k 10 200 python -u tools/root_probe.py $S > "$O/root_256.log" 2>&1
rc=$?; echo "256 rc=$rc"; grep -v -e Warn -e amdgpu.ids "$O/root_256.log"; exit $rc
