#!/bin/bash
# Round 4, session 15: fp32 GEMM variants on C5's 1x1 add-on GEMM (M=16384, N=2048, K=192) and
# the split-bf16 PMC pass (alt_precision's roofline traffic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s15
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
LAB_VARIANTS=0,1,2,3,4,5,7,8 LAB_GROUPS=1,4,8,16 LAB_SHAPES=c5_addon LAB_ROUNDS=5 timeout -k 10 300 python tools/gemm_lab.py > $O/lab_addon.log 2>&1; step lab $?
grep -v "amdgpu.ids" $O/lab_addon.log
PMC_OUT=pmc_s3 PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra --precision bf16x3 --alt-precision none --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > $O/pmc_s3.log 2>&1; step pmc $?
tail -6 $O/pmc_s3.log
