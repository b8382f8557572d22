#!/bin/bash
# Round 4, session 13: quad-layout bf16 head (whole-line proto stores): test + C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s13
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "head_bf16_quad" -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 400 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.head_bf16_quads:0:1 c3 --rounds 7 > $O/ab_c3_head.txt 2>&1; step abc3 $?
grep "^{" $O/ab_c3_head.txt
