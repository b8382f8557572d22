#!/bin/bash
# Round 4, session 32: where the fp32 GEMM's vector epilogue spends its cycles -- per store
# iteration of the first 32-row slab (lab stamps 12-15, variant 30 = the product tile stamped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s32
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
timeout -k 10 300 python tools/gemm_stamps.py s384_fc1,s768_fc1,s384_fc2 > $O/stamps_epi.txt 2>&1; step stamps $?
cat $O/stamps_epi.txt
