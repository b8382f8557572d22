#!/bin/bash
# Round 4 PMC passes on the tree after the epilogue wait-count fix (sources changed -> new digests):
# r4_pmc.sh (C2, C3, C5) plus the split-bf16 C2 pass of r4_s15.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/pmc_all.sh || exit $?
PMC_OUT=pmc_s3 PMC_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-extra --precision bf16x3 --alt-precision none --stream-split 1" \
  timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc_s3.log 2>&1 || exit $?
tail -6 gpurun_out/pmc_s3.log
echo "r4 pmc2 done"
