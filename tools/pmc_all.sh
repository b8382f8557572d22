#!/bin/bash
# PMC passes (clock / MFMA busy, FETCH_SIZE, WRITE_SIZE; separate runs) over C2 (bench.py),
# C3 and C5 (tools/bench_configs.py), one stream each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra --alt-precision none --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
tail -8 gpurun_out/pmc.log
PMC_OUT=pmc_c3 PMC_TARGET=tools/bench_configs.py PMC_ARGS="--only c3 --steps 3 --warmup 1 --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_c3.log 2>&1 || exit $?
tail -8 gpurun_out/pmc_c3.log
PMC_OUT=pmc_c5 PMC_TARGET=tools/bench_configs.py PMC_ARGS="--only c5 --steps 3 --warmup 1 --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_c5.log 2>&1 || exit $?
tail -8 gpurun_out/pmc_c5.log
echo "r4 pmc done"
