#!/bin/bash
# Round 5: bf16 raster group budget A/B (PIPNET_BF16_GROUP_BUDGET 2 MiB product vs 1 / 0.5 MiB builds),
# C3 end to end, three interleaved rounds of separate processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/ab_group.txt
: > $out
for r in 1 2 3; do
  for v in product g1m g05m; do
    if [ $v = product ]; then lib=count_pipnet_amd/libpipnet_amd.so; else lib=tools/ab/libpipnet_$v.so; fi
    PIPNET_AMD_LIB=$PWD/$lib timeout -k 10 180 python tools/bench_configs.py --only c3 --steps 20 > gpurun_out/ab_group_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "arm $v failed rc=$rc" >> $out; exit $rc; }
    echo "round $r $v $(grep '^{' gpurun_out/ab_group_$v.log | head -1 | cut -c1-200)" >> $out
  done
done
cat $out
