#!/bin/bash
# Round 4, session 9: direct epilogue with plain (not non-temporal) stores.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s9
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "direct_epilogue" -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 300 python tools/c3_diag.py --tiles 9 --ds 0,1 --reps 20 --only l3.c1,l4.c1,l3.c3,l4.ds,l4.c3 > $O/c3_diag_ds.log 2>&1; step c3diag $?
grep -v "amdgpu.ids" $O/c3_diag_ds.log
