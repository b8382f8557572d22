#!/bin/bash
# Round 4, session 34: epilogue wait-count fix (vm_drain after the bias / residual preloads, fp32
# slab reads hoisted, MLP epilogue loads before its stores).  GPU suite on the new library, then
# bench.py alternating the previous library (ablib/, PIPNET_AMD_LIB) and the new one, twice.
# (ablib/libpipnet_amd_base.so was a copy of the library built from the previous commit; removed after the run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s34
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt; step pytest $rc
for r in 1 2; do
  PIPNET_AMD_LIB=$R/ablib/libpipnet_amd_base.so PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 400 python bench.py --no-cpu-baseline > $O/base_$r.log 2>&1; step base$r $?
  timeout -k 10 400 python bench.py --no-cpu-baseline > $O/new_$r.log 2>&1; step new$r $?
  for f in base_$r new_$r; do
    python -c "
import json,sys
d=json.loads(open('$O/$f.log').read().strip().split('\n')[-1])
print('$f', round(d['value'],1), round(d['extra']['c3']['value'],1), round(d['extra']['c5']['value'],1), round(d.get('alt_precision',{}).get('value',0),1), 'C2frac', round(d['roofline']['frac'],4), 'C3frac', round(d['extra']['c3']['roofline']['frac'],4))"
  done
done
