#!/bin/bash
# Round 4, session 7: four-wave 256x256 bf16 tile with AGPR-pinned accumulators (lab) vs the
# product ping-pong tile and hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s7
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 200 python tools/bf16_lab.py --build-only > $O/build.log 2>&1; step build $?
LAB_ABL=0,1040,2,1042,-1 LAB_SHAPES=sq4096,l4ds,l4c1,l3c3,l3c1,sq8192 LAB_ROUNDS=3 timeout -k 10 400 python tools/bf16_lab.py > $O/q4a.log 2>&1; step q4a $?
grep -v "amdgpu.ids" $O/q4a.log
