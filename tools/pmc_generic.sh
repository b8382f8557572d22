#!/bin/bash
# Generic PMC passes: PMC_SETS="ctrA ctrB;ctrC;..." (one rocprofv3 --kernel-trace --pmc run per
# set, as MI355X_MICROARCH.md prescribes), over PMC_CMD (a python script + args, run from the
# repo root).  Prints per-kernel mean of every counter (tools/pmc_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT="$R/gpurun_out/${PMC_OUT:-pmcg}"
mkdir -p "$OUT"
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${PMC_SETS}"
i=0
for ctr in "${SETS[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/p$i" -o run --output-format csv -- python3 $R/$PMC_CMD > "$OUT/p$i.log" 2>&1)
  rc=$?
  echo "[pmc pass $i: $ctr] exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
python3 tools/pmc_table.py "$OUT" > "$OUT/table.txt" 2>&1; cat "$OUT/table.txt"
