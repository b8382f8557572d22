#!/bin/bash
# Round 4, session 2: fp32 GEMM 2- vs 3-workgroup-per-CU tiles on the stage-3/4 shapes (lab),
# their stamps, and the hipBLASLt kernels torch picks for the C3 1x1 shapes (names = tile config).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4d2
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
LAB_VARIANTS=0,7,8 LAB_GROUPS=8 LAB_SHAPES=s384_fc1,s384_fc2,s768_fc1,s768_fc2 timeout -k 10 300 python tools/gemm_lab.py > $O/lab.log 2>&1; step lab $?
grep -v "^\[\|amdgpu.ids" $O/lab.log
STAMP_VAR=37 timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1 > $O/stamps_v7.log 2>&1; step stamps7 $?
timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1 > $O/stamps_v0.log 2>&1; step stamps0 $?
grep -v "amdgpu.ids" $O/stamps_v7.log $O/stamps_v0.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/libk -o run --output-format csv -- python3 $R/tools/c3_diag.py --tiles 9 --reps 5 > $O/libk.log 2>&1); step libk $?
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r4d2/libk/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in rows:
    print(r.get("Name", "")[:200], r.get("Calls"), r.get("AverageNs"))
PY
