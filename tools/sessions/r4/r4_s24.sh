#!/bin/bash
# Round 4, session 24: interleaved sub-batch enqueue with the first sub-batch k blocks ahead.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s24
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 500 python tools/ab_toggle.py fn:count_pipnet_amd.pipnet.set_interleave_lag:0:1:2:4:8 c3 --rounds 5 > $O/ab_c3_lag.txt 2>&1; step c3 $?
grep "^{" $O/ab_c3_lag.txt
timeout -k 10 600 python tools/ab_toggle.py fn:count_pipnet_amd.pipnet.set_interleave_lag:0:2:6:12 c2 --rounds 5 > $O/ab_c2_lag.txt 2>&1; step c2 $?
grep "^{" $O/ab_c2_lag.txt
