#!/bin/bash
# Round 4, session 6: fp32 GELU epilogue forms (lab), the restructured staggered MLP (lab), bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s6
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
LAB_VARIANTS=0 LAB_GROUPS=8 LAB_EPIS=2,102,103,100,1 LAB_SHAPES=s384_fc1,s768_fc1 LAB_ROUNDS=5 timeout -k 10 300 python tools/gemm_lab.py > $O/lab_gelu.log 2>&1; step labgelu $?
grep -v "^\[\|amdgpu.ids" $O/lab_gelu.log
LAB_ROUNDS=5 timeout -k 10 400 python tools/mlp_lab.py > $O/mlp_lab.log 2>&1; step mlplab $?
grep "^{" $O/mlp_lab.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; step bench $?
tail -1 $O/bench.log | cut -c1-400
