#!/bin/bash
# round-3 GPU session: changed tests, streaming-GEMM A/B, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_stream or gemm_persistent" > gpurun_out/r3_stream_tests.log 2>&1
rc=$?; echo "stream tests rc $rc"; tail -5 gpurun_out/r3_stream_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ $rc -ne 0 ] && exit 1
for i in 1 2; do
  for mode in 0 1; do
    PIPNET_GEMM_STREAM=$mode timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r3_gemm_stream$mode.$i.log 2>&1 || exit $?
    echo "stream=$mode run $i"; grep -v "^\[\|amdgpu" gpurun_out/r3_gemm_stream$mode.$i.log | head -9
  done
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py tests/test_gpu_bf16.py tests/test_bench_harness.py "tests/test_gpu_train.py::test_finetune_iterations_match_reference" "tests/test_gpu_train.py::test_suffix_training_matches_reference" -s > gpurun_out/r3_tests1.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "passed|failed|PASSED|FAILED|budget|running statistics" gpurun_out/r3_tests1.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3_bench1.log 2>&1; rc=$?; echo "bench rc $rc"; tail -c 4000 gpurun_out/r3_bench1.log
exit $rc
