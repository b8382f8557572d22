#!/bin/bash
# streaming fp32 GEMM: bitwise tests, then interleaved A/B against the regular tile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_stream or gemm_persistent or linear" > gpurun_out/r3_stream_tests.log 2>&1
rc=$?; echo "stream tests rc $rc"; tail -4 gpurun_out/r3_stream_tests.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for mode in 0 1; do
    PIPNET_GEMM_STREAM=$mode timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r3_gemm_stream$mode.$i.log 2>&1 || exit $?
    echo "stream=$mode run $i"; grep -v "^\[\|amdgpu" gpurun_out/r3_gemm_stream$mode.$i.log | head -9 | tail -4
  done
done
