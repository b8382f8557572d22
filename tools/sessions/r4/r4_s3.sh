#!/bin/bash
# Round 4, session 3: 224-row ping-pong tiles (RB = 7) -- bitwise tests, per-layer and end-to-end
# C3 A/B -- plus the fp32 GEMM 3-workgroup lab and the hipBLASLt kernel names for the C3 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s3
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ] && [ "$2" -ne 1 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -3 $O/pt.log
timeout -k 10 300 python tools/c3_diag.py --tiles 9 --rb 8,7 --only l3.c1,l4.c1,l3.c3,l4.ds,l4.c3 > $O/c3_diag_rb.log 2>&1; step c3diag $?
grep -v "^\[\|amdgpu.ids" $O/c3_diag_rb.log
timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --rb-ab --reps 20 > $O/conv_rb_ab.log 2>&1; step convab $?
grep -v "^\[\|amdgpu.ids" $O/conv_rb_ab.log
timeout -k 10 300 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_rb:8:0 c3 --rounds 6 > $O/ab_c3_rb.log 2>&1; step abc3 $?
grep "^{" $O/ab_c3_rb.log
LAB_VARIANTS=0,7,8 LAB_GROUPS=8 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2 timeout -k 10 300 python tools/gemm_lab.py > $O/lab.log 2>&1; step lab $?
grep -v "^\[\|amdgpu.ids" $O/lab.log
STAMP_VAR=37 timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1 > $O/stamps_v7.log 2>&1; step stamps7 $?
grep -v "amdgpu.ids" $O/stamps_v7.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/libk -o run --output-format csv -- python3 $R/tools/c3_diag.py --tiles 9 --reps 3 --only l3.c1,l4.c1,l4.ds,l3.c3,sq8k > $O/libk.log 2>&1); step libk $?
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r4s3/libk/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "Cijk" in r.get("Name", "") or "ppp" in r.get("Name", ""):
            print(r.get("Name", "")[:230], r.get("Calls"), r.get("AverageNs"))
PY
