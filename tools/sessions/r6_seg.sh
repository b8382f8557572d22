#!/bin/bash
# Round 6: SEG 3 (one 32-MFMA segment per K-tile, product) vs SEG 2 (tools/ab/libpipnet_seg2.so) on the bf16
# ping-pong tiles: bitwise digests of both builds, the bf16 GPU tests on the product, then interleaved C3 timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/seg_ab.txt
: > $out
for v in product seg2; do
  lib=$R/count_pipnet_amd/libpipnet_amd.so; [ $v = product ] || lib=$R/tools/ab/libpipnet_$v.so
  PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=$lib timeout -k 10 200 python tools/bf16_digest.py > gpurun_out/digest_$v.log 2>&1
  rc=$?; echo "digest $v $(grep '^{' gpurun_out/digest_$v.log)" >> $out; [ $rc -eq 0 ] || { tail -20 gpurun_out/digest_$v.log; exit $rc; }
done
cat $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_bf16.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_bf16.txt; [ $rc -eq 0 ] || exit $rc
ARMS="product seg2" CFG=c3 ROUNDS=${ROUNDS:-3} LAYERS=${LAYERS:-l3.c2,l4.c2,l3.c3,l4.c3,l3.c1,l4.c1,l2.ds} bash tools/sessions/r5_ab.sh
