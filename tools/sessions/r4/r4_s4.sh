#!/bin/bash
# Round 4, session 4: end-to-end A/B of the 224-row ping-pong tiles per kernel (C3, default and one
# stream), the 3-workgroup fp32 tile on C2, and the fp32 epilogue (lab ablation + sub-phase stamps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s4
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_rb:8:0:1:2 c3 --rounds 8 > $O/ab_c3_rb.log 2>&1; step abc3 $?
grep "^{" $O/ab_c3_rb.log
timeout -k 10 300 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_rb:8:0 c3 --rounds 6 --stream-split 1 > $O/ab_c3_rb_s1.log 2>&1; step abc3s1 $?
grep "^{" $O/ab_c3_rb_s1.log
timeout -k 10 300 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.gemm_bk16x3:0:1 c2 --rounds 8 > $O/ab_c2_bk16x3.log 2>&1; step abc2 $?
grep "^{" $O/ab_c2_bk16x3.log
LAB_VARIANTS=0,8 LAB_GROUPS=8 LAB_EPIS=2,1,0 LAB_SHAPES=s384_fc1,s768_fc1 timeout -k 10 300 python tools/gemm_lab.py > $O/lab_epi.log 2>&1; step labepi $?
grep -v "^\[\|amdgpu.ids" $O/lab_epi.log
timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1 > $O/stamps_v0.log 2>&1; step stamps0 $?
grep -v "amdgpu.ids" $O/stamps_v0.log
