#!/bin/bash
# Round 5: end-to-end A/B of library builds (product vs tools/ab/libpipnet_<arm>.so) on one BASELINE config,
# interleaved rounds of separate processes.  ARMS="product before" CFG=c3 ROUNDS=3 [LAYERS=l3.c3,l4.c3] [EXTRA="--stream-split 1"]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
ARMS=${ARMS:-"product before"}; CFG=${CFG:-c3}; ROUNDS=${ROUNDS:-3}
out=gpurun_out/ab_${CFG}.txt
: > $out
lib_of() { if [ $1 = product ]; then echo $R/count_pipnet_amd/libpipnet_amd.so; else echo $R/tools/ab/libpipnet_$1.so; fi; }
for r in $(seq $ROUNDS); do
  for v in $ARMS; do
    PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$(lib_of $v) timeout -k 10 180 python tools/bench_configs.py --only $CFG --steps 20 ${EXTRA:-} > gpurun_out/ab_${CFG}_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$CFG arm $v failed rc=$rc" >> $out; tail -5 gpurun_out/ab_${CFG}_$v.log >> $out; exit $rc; }
    echo "$CFG round $r $v $(grep '^{' gpurun_out/ab_${CFG}_$v.log | head -1 | cut -c1-100)" >> $out
  done
done
if [ -n "${LAYERS:-}" ]; then
  for v in $ARMS; do
    echo "== layers $v" >> $out
    PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$(lib_of $v) timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --only $LAYERS --tiles -1 --rotate 4 2>&1 | grep -v "^\[\|amdgpu.ids" >> $out
    rc=$?; [ $rc -eq 0 ] || exit $rc
  done
fi
cat $out
