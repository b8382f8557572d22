#!/bin/bash
# Round 4, session 11: do the two fp32 GEMM workgroups of a CU run their epilogues at the same
# time?  (tools/gemm_stamps.py epilogue coincidence)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s11
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python tools/gemm_stamps.py s384_fc1,s384_fc2,s768_fc1,s768_fc2,s192_fc1 > $O/stamps.log 2>&1; step stamps $?
grep -v "amdgpu.ids" $O/stamps.log
