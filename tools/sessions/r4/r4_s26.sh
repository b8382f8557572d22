#!/bin/bash
# Round 4, session 26: fused CNBlock MLP with three LDS stages (weight chunk two ahead).
# (lab variants 51-53 and the NSTG template parameter were removed after this run: profiles/r04/mlp_nstg3_lab.txt)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s26
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
LAB_VARIANTS='{"96": [0, 51], "192": [0, 21, 52, 53]}' LAB_ROUNDS=7 timeout -k 10 400 python tools/mlp_lab.py > $O/mlp_nstg3.txt 2>&1; step lab $?
cat $O/mlp_nstg3.txt
