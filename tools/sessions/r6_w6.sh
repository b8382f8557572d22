#!/bin/bash
# Round 6: 96 x 384 BK16 tile at 2 per CU on the GELU fc1 shapes (lab rule 10) -- per-shape timing through the product entry
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/w6.txt
: > $out
for v in product w6 product w6; do
  if [ $v = product ]; then L=$R/count_pipnet_amd/libpipnet_amd.so; else L=$R/tools/ab/libpipnet_$v.so; fi
  echo "== gemm $v" >> $out
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$L timeout -k 10 240 python tools/vendor_f32_gemm.py 2>&1 | grep '^{' | cut -c1-110 >> $out
  rc=$?; [ $rc -eq 0 ] || { cat $out; exit $rc; }
done
cat $out
