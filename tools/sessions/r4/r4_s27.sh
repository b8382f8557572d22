#!/bin/bash
# Round 4, session 27: fused CNBlock MLP with the weight fragments of the next group read ahead
# of the current group's MFMAs (PF 1: GEMM1, 2: GEMM2, 3: both; sched_barrier keeps the order).
# (lab variants 61-65 and the PF template parameter were removed after this run: profiles/r04/mlp_prefetch_lab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s27
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
LAB_VARIANTS='{"96": [0, 61, 64, 65], "192": [0, 21, 62, 63]}' LAB_ROUNDS=7 timeout -k 10 400 python tools/mlp_lab.py > $O/mlp_pf.txt 2>&1; step lab $?
cat $O/mlp_pf.txt
