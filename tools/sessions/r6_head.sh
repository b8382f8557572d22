#!/bin/bash
# Round 6: NonNegLinear as a per-wave GEMV (both head paths), fused head's tail spread over the waves --
# head tests, then FUSED_HEAD off / on on C2 and C3 (tools/ab_toggle.py, interleaved in one process),
# then a kernel-stats pass of C2 (two-kernel head) for the nonneg_linear_kernel time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/head.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "head or nonneg or softmax_pool" > gpurun_out/head_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/head_tests.txt >> $out; [ $rc -eq 0 ] || { cat $out; tail -30 gpurun_out/head_tests.txt; exit $rc; }
for c in c2 c3; do
  timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.FUSED_HEAD $c --rounds 5 > gpurun_out/head_ab_$c.log 2>&1
  rc=$?; grep '^{' gpurun_out/head_ab_$c.log >> $out; [ $rc -eq 0 ] || { tail -5 gpurun_out/head_ab_$c.log; exit $rc; }
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run --output-format csv \
  -- python tools/bench_configs.py --only c2 --steps 10 > gpurun_out/prof_head.log 2>&1 || exit $?
grep -h "nonneg\|softmax_pool" gpurun_out/prof_head/*kernel_stats.csv gpurun_out/prof_head/*/*kernel_stats.csv 2>/dev/null | cut -c1-200 >> $out
cat $out
