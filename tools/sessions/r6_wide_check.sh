#!/bin/bash
# Round 6: the wide fp32 tile in the product -- its bitwise / bounds tests, then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "wide or product_tile or gemm" > gpurun_out/wide_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/wide_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_suite.txt 2>&1
rc=$?; tail -3 gpurun_out/wide_suite.txt; exit $rc
