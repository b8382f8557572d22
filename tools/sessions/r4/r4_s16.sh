#!/bin/bash
# Round 4, session 16: stream splits re-checked on the round-4 kernels (C2 2/3, C5 1/2, C3 2/3),
# then the C5 PMC passes (MLP kernel names changed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s16
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python tools/ab_toggle.py streams:2:3 c2 --rounds 5 > $O/ab_c2_streams.txt 2>&1; step c2 $?
grep "^{" $O/ab_c2_streams.txt
timeout -k 10 300 python tools/ab_toggle.py streams:1:2 c5 --rounds 7 --steps 30 > $O/ab_c5_streams.txt 2>&1; step c5 $?
grep "^{" $O/ab_c5_streams.txt
timeout -k 10 400 python tools/ab_toggle.py streams:2:3 c3 --rounds 5 > $O/ab_c3_streams.txt 2>&1; step c3 $?
grep "^{" $O/ab_c3_streams.txt
PMC_OUT=pmc_c5 PMC_TARGET=tools/bench_configs.py PMC_ARGS="--only c5 --steps 3 --warmup 1 --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > $O/pmc_c5.log 2>&1; step pmc $?
tail -4 $O/pmc_c5.log
