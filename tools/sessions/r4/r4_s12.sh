#!/bin/bash
# Round 4, session 12: fp32 GEMM output tiles with plain (cached) vs non-temporal stores, end to
# end on C2 and C5 (the next kernel reads the tile: Infinity Cache vs HBM).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s12
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.gemm_plain_store:0:1 c2 --rounds 5 > $O/ab_c2.txt 2>&1; step abc2 $?
grep "^{" $O/ab_c2.txt
timeout -k 10 300 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.gemm_plain_store:0:1 c5 --rounds 7 --steps 30 > $O/ab_c5.txt 2>&1; step abc5 $?
grep "^{" $O/ab_c5.txt
