#!/bin/bash
# Round 4, session 31: re-test the three-workgroups-per-CU BK16 tiles (lab v7 = <16,2,3,3>,
# v8 = <16,2,3,2>) against the product tile (v0) on the stage-3/4 fc1 / fc2 shapes, 9 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s31
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
# the lab library is gpurun-ignored: build it on the box
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
LAB_VARIANTS=0,7,8 LAB_GROUPS=8 LAB_ROUNDS=9 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2,s192_fc1,s192_fc2 \
  timeout -k 10 500 python tools/gemm_lab.py > $O/gemm_3wg.txt 2>&1; step lab $?
cat $O/gemm_3wg.txt
