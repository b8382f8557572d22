#!/bin/bash
# Round 4, first GPU session: bf16 1x1 tile vs hipBLASLt (quantisation vs per-CU efficiency),
# and the fp32 GEMM clock reconciliation (stamps and GRBM_GUI_ACTIVE on the same dispatches).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4d1
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread -k "f64acc or fold_tracks" > $O/pt_fold.log 2>&1; step ptfold $?
tail -3 $O/pt_fold.log
timeout -k 10 300 python tools/c3_diag.py > $O/c3_diag.log 2>&1; step c3diag $?
grep -v "^\[\|amdgpu.ids" $O/c3_diag.log
timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1,s768_fc2 > $O/clk0.log 2>&1; step stamps $?
PMC="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --pmc $PMC -d $O/clk1 -o run --output-format csv -- python3 $R/tools/gemm_stamps.py s384_fc1,s384_fc2,s768_fc1,s768_fc2 > $O/clk1.log 2>&1); step pmc1 $?
(cd /tmp && STAMP_MSCALE=12 timeout -k 10 240 rocprofv3 --kernel-trace --pmc $PMC -d $O/clk2 -o run --output-format csv -- python3 $R/tools/gemm_stamps.py s384_fc1,s768_fc1 > $O/clk2.log 2>&1); step pmc2 $?
python tools/clock_reconcile.py $O/clk1 $O/clk1.log > $O/reconcile.txt 2>&1
python tools/clock_reconcile.py $O/clk2 $O/clk2.log >> $O/reconcile.txt 2>&1
cat $O/reconcile.txt
grep "clk=" $O/clk0.log
