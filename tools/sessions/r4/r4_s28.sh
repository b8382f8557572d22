#!/bin/bash
# Round 4, session 28: sub-batch stream counts with the interleaved enqueue (C3, C2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s28
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python tools/ab_toggle.py streams:2:3:4 c3 --rounds 6 > $O/ab_c3_streams.txt 2>&1; step c3 $?
grep "^{" $O/ab_c3_streams.txt
timeout -k 10 500 python tools/ab_toggle.py streams:2:3 c2 --rounds 5 > $O/ab_c2_streams.txt 2>&1; step c2 $?
grep "^{" $O/ab_c2_streams.txt
