#!/bin/bash
# Round 4, session 8: direct (register) epilogue of the persistent 1x1 bf16 tile -- bitwise test,
# per-layer timing vs the LDS epilogue and hipBLASLt, C3 end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s8
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "direct_epilogue or 224_rows" -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -3 $O/pt.log
timeout -k 10 300 python tools/c3_diag.py --tiles 9 --ds 0,1 --reps 20 > $O/c3_diag_ds.log 2>&1; step c3diag $?
grep -v "amdgpu.ids" $O/c3_diag_ds.log
timeout -k 10 400 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_direct_epi:0:1 c3 --rounds 5 > $O/ab_c3_ds.txt 2>&1; step abc3 $?
grep "^{" $O/ab_c3_ds.txt
