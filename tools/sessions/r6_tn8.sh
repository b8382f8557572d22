#!/bin/bash
# Round 6: the 8-wave 256-row fp32 GEMM tile (gemm_f32.hip variant 4) -- GEMM GPU tests, per-shape timing
# against the vendor GEMM, then C2 end to end: product vs tn4 (the same sources built with the rule off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "8wave or product_tile or splitk or gemm" > gpurun_out/tn8_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/tn8_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vendor_f32_gemm.py > gpurun_out/tn8_vendor.txt 2>&1 || exit $?
cat gpurun_out/tn8_vendor.txt
ARMS="product tn4" CFG=c2 ROUNDS=${ROUNDS:-4} bash tools/sessions/r5_ab.sh
