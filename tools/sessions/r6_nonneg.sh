#!/bin/bash
# Round 6: the two-kernel head's NonNegLinear (4 slices per unrolled step) -- head tests, then its kernel time in
# C5 / C2 / C3 (rocprofv3 --stats, one stream).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c5.py -x -q --timeout 120 --timeout-method thread \
  -k "head or nonneg or softmax_pool or count" > gpurun_out/nonneg_tests.txt 2>&1
rc=$?; tail -1 gpurun_out/nonneg_tests.txt; [ $rc -eq 0 ] || { tail -30 gpurun_out/nonneg_tests.txt; exit $rc; }
export TMPDIR=/tmp
for c in c5 c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_nn_$c -o run --output-format csv \
    -- python tools/bench_configs.py --only $c --steps 10 --stream-split 1 > gpurun_out/prof_nn_$c.log 2>&1 || exit $?
  echo "== $c"; grep -h "nonneg" gpurun_out/prof_nn_$c/run_kernel_stats.csv | cut -c1-160
done
