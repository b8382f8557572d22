#!/bin/bash
# Round 6: BK16 128-row tiles at 3 per CU on K <= 768 (lab rule 8) -- per-shape timing through the product entry
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/bk16m3.txt
: > $out
for v in product bk16m3 product bk16m3; do
  if [ $v = product ]; then L=$R/count_pipnet_amd/libpipnet_amd.so; else L=$R/tools/ab/libpipnet_$v.so; fi
  echo "== gemm $v" >> $out
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$L timeout -k 10 240 python tools/vendor_f32_gemm.py 2>&1 | grep '^{' | cut -c1-110 >> $out
  rc=$?; [ $rc -eq 0 ] || { cat $out; exit $rc; }
done
cat $out
echo "== ab_toggle FUSED_MLP c2" >> $out
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.convnext_features.FUSED_MLP c2 --rounds 5 2>&1 | grep '^{\|bitwise' >> $out || exit $?
tail -8 $out
