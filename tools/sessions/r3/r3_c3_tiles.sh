#!/bin/bash
# C3 tile-rule change: bf16 tests, per-layer bench (auto choice), C3 throughput
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_graph.py "tests/test_gpu_parity.py::test_hip_forward_matches_reference_golden" -s > gpurun_out/r3_c3t.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r3_c3t.log; grep -E "FAILED|^E  |budget" gpurun_out/r3_c3t.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --tiles=-1 > gpurun_out/r3_conv_b64_auto.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/r3_conv_b64_auto.log
for r in 1 2; do
  timeout -k 10 200 python tools/bench_configs.py --only c3 --steps 30 --warmup 5 > gpurun_out/r3_c3_$r.log 2>&1 || exit $?
  grep "^{" gpurun_out/r3_c3_$r.log
done
