#!/bin/bash
# Round 4, session 33: the fp32 GEMM vector epilogue's per-store vmcnt(0) (hipcc's wait-count pass
# cannot count stores issued inside the row-guard branches, so it waits for every earlier store
# before each bias / residual use).  v50 / v52: one explicit vmcnt(0) before the store loop;
# v54 / v56: + the slab's 8 LDS reads hoisted out of the branches.  v0 / v2 = product tiles.
# (lab variants 50-56 / ABL bits 16, 32 were folded into the product epilogue after this run: profiles/r04/epilogue_vmcnt_ab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s33
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
LAB_VARIANTS=0,50,54,2,52,56 LAB_GROUPS=8 LAB_ROUNDS=7 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2,c5_addon \
  timeout -k 10 500 python tools/gemm_lab.py > $O/gemm_vmcnt.txt 2>&1; step lab $?
cat $O/gemm_vmcnt.txt
