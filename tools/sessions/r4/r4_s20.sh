#!/bin/bash
# Round 4, session 20: do the conv3 + identity layer rankings (persistent ping-pong tile vs the
# two-workgroup tile 4) flip once the bench's buffers rotate beyond the Infinity Cache?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s20
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for rot in 1 4; do
  timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --tiles=-1,4 --reps 20 --rotate $rot --only l1.c3,l2.c3,l3.c3,l4.c3,l3.c1 > $O/rot$rot.log 2>&1; step rot$rot $?
  echo "rotate $rot"; grep -v amdgpu.ids $O/rot$rot.log
done
