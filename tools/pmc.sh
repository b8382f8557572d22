#!/bin/bash
# PMC passes (separate runs, kernel-trace only, as MI355X_MICROARCH.md prescribes) over the
# bench workload: clock + MFMA busy, then HBM read bytes, then HBM write bytes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/${PMC_OUT:-pmc}
mkdir -p $O
export TMPDIR=/tmp
CMD="python3 $R/${PMC_TARGET:-bench.py} ${PMC_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}"
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d "$R/$O/p$i" -o run --output-format csv -- $CMD > "$R/$O/p$i.log" 2>&1)
  rc=$?
  echo "[pmc pass $i: $ctr] exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "$R/$O/p$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
