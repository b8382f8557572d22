#!/bin/bash
# Round 4, session 17: tile 12 (128x128, 3 stages, 3 workgroups / CU) -- bitwise test, per-layer
# timing against the automatic tiles at 64 images (one C3 stream).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s17
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "tile12" -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --tiles=-1,4,12,0 --reps 20 > $O/conv_t12.log 2>&1; step bench $?
grep -v amdgpu.ids $O/conv_t12.log
timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --tiles=-1,4,12,0 --reps 20 --only l1.c1,l1.c3,l2.c1,l2.c2s2,l2.ds,l2.c2 > $O/conv_t12b.log 2>&1; step bench2 $?
grep -v amdgpu.ids $O/conv_t12b.log
