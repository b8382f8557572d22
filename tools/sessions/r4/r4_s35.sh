#!/bin/bash
# Round 4, session 35: the per-store-iteration epilogue stamps of session 32 re-run after the
# wait-count fix (variant 30 / 32 = the product tiles stamped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s35
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2> $O/build.txt; step build $?
timeout -k 10 300 python tools/gemm_stamps.py s384_fc1,s768_fc1,s384_fc2 > $O/stamps_epi.txt 2>&1; step stamps $?
cat $O/stamps_epi.txt
