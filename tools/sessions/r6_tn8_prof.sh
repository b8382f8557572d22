#!/bin/bash
# Round 6: per-kernel times of C2 with the product library vs tn4 (variant 4 off), rocprofv3 --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in product tn4; do
  if [ $v = product ]; then L=$R/count_pipnet_amd/libpipnet_amd.so; else L=$R/tools/ab/libpipnet_$v.so; fi
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run --output-format csv \
    -- python tools/bench_configs.py --only c2 --steps 10 ${EXTRA:-} > gpurun_out/prof_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_$v.log; exit $rc; }
done
for v in product tn4; do
  f=$(ls gpurun_out/prof_$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/prof_$v/run_kernel_stats.csv)
  echo "== $v"; head -14 $f | cut -c1-220
done
