#!/bin/bash
# Round 6: the wide 192 x 384 fp32 tile (gemm_f32.hip variant 5, built with -DPIPNET_AB_GEMM_RULE=5 as
# tools/ab/libpipnet_wide.so): bitwise digests vs the product, per-shape timing through the product
# entry, C2 end to end interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/wide.txt
: > $out
for v in product wide; do
  if [ $v = product ]; then L=$R/count_pipnet_amd/libpipnet_amd.so; else L=$R/tools/ab/libpipnet_$v.so; fi
  echo "== digest $v" >> $out
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$L timeout -k 10 240 python tools/f32_digest.py > gpurun_out/wide_dig_$v.log 2>&1
  rc=$?; grep '^{' gpurun_out/wide_dig_$v.log >> $out; [ $rc -eq 0 ] || { tail -5 gpurun_out/wide_dig_$v.log >> $out; cat $out; exit $rc; }
done
for v in product wide product wide; do
  if [ $v = product ]; then L=$R/count_pipnet_amd/libpipnet_amd.so; else L=$R/tools/ab/libpipnet_$v.so; fi
  echo "== gemm $v" >> $out
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$L timeout -k 10 240 python tools/vendor_f32_gemm.py 2>&1 | grep '^{' | cut -c1-120 >> $out
  rc=$?; [ $rc -eq 0 ] || { cat $out; exit $rc; }
done
cat $out
ARMS="product wide" CFG=c2 ROUNDS=${ROUNDS:-4} bash tools/sessions/r5_ab.sh
