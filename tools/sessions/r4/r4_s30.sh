#!/bin/bash
# Round 4, session 30: fp32 GEMM wave priorities -- main loop at s_setprio 1 (the partner's
# epilogue VALU yields to the MFMA stream) or epilogue at s_setprio 2 -- vs the product tile.
# (lab variants 50-53 and ABL bits 32 / 64 were removed after this run: profiles/r04/gemm_setprio.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s30
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
# the lab library is gpurun-ignored: build it on the box
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
LAB_VARIANTS=0,50,51,2,52,53 LAB_GROUPS=8 LAB_ROUNDS=7 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2 \
  timeout -k 10 500 python tools/gemm_lab.py > $O/gemm_prio.txt 2>&1; step lab $?
cat $O/gemm_prio.txt
