#!/bin/bash
# Round 4, session 14: dwconv7 + LN with the LayerNorm in registers (lab v50-v53) vs the
# round-4 product tiles (v40-v43) and TY = 1 (v0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s14
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
DW_VARIANTS=0,40,41,42,43,50,51,52,53 DW_SHAPES=96x56,192x28,384x27,768x26,96x32,192x16 timeout -k 10 400 python tools/dw_lab.py > $O/dw_lnr.log 2>&1; step dwlab $?
grep -v amdgpu.ids $O/dw_lnr.log
