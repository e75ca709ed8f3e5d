#!/bin/bash
# round 2, call AE: A/B diagnostics (HEAD build vs current code) of the root's first checks and warm children
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02ae; mkdir -p $O
for v in head cur; do
  L=neptune-mip_amd/lib/variants/libneptune_lp_$v.so; [ $v = cur ] && L=neptune-mip_amd/lib/libneptune_lp.so
  NEPTUNE_LP_LIB=$PWD/$L timeout -k 10 200 python -u tools/ab_probe.py > $O/p_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v "amdgpu\|Initializ" $O/p_$v.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
done
