#!/bin/bash
# Round 4, session 21: sub-batch streams with priorities (first stream high) vs equal priority.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s21
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.STREAM_PRIORITY c2 --rounds 7 > $O/ab_c2_prio.txt 2>&1; step c2 $?
grep "^{" $O/ab_c2_prio.txt
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.STREAM_PRIORITY c3 --rounds 7 > $O/ab_c3_prio.txt 2>&1; step c3 $?
grep "^{" $O/ab_c3_prio.txt
