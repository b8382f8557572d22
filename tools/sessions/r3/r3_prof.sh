#!/bin/bash
# round-3 evidence: rocprofv3 kernel stats of the default bench run, then the PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --stream-split 1 > "$R/gpurun_out/prof_bench.log" 2>&1) || exit $?
tail -c 1500 gpurun_out/prof_bench.log
PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra --alt-precision none --stream-split 1" timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1 || exit $?
tail -25 gpurun_out/pmc.log
