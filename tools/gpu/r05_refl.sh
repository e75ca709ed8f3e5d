#!/bin/bash
# Round 5: the NEP_INLINE_REFLECT build (lib/variants/libneptune_lp_refl.so): the whole -m gpu suite on it, then
# the replay bench A/B against the default build
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05_refl}; mkdir -p "$O"
export TMPDIR=/tmp
NEPTUNE_LP_LIB=$PWD/neptune-mip_amd/lib/variants/libneptune_lp_refl.so timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_refl.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$O/pytest_refl.log"; grep FAILED "$O/pytest_refl.log" | head; [ $rc -le 1 ] || exit $rc
bash tools/gpu/r05_ab.sh "${1:-r05_refl}" lib/variants/libneptune_lp_refl.so
