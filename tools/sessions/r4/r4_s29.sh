#!/bin/bash
# Round 4, session 29: fp32 GEMM epilogue with wave-local slab sync (lab ABL 16: one workgroup
# barrier instead of two per 32-row block) vs the product tile, on the C2 stage-3/4 shapes.
# (lab variants 50 / 52 / 80 and ABL bit 16 were removed after this run: profiles/r04/gemm_epilogue_wavesync.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s29
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
# the lab library is gpurun-ignored: build it on the box
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
LAB_VARIANTS=0,50,2,52 LAB_GROUPS=8 LAB_ROUNDS=7 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2,s192_fc1 \
  timeout -k 10 500 python tools/gemm_lab.py > $O/gemm_wavesync.txt 2>&1; step lab $?
cat $O/gemm_wavesync.txt
