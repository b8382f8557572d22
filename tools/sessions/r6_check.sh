#!/bin/bash
# Round 6 check on one GPU box: the new Philox parity tests first, then the whole GPU suite, then the
# default bench line (no CPU baseline).  Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ "${SKIP_PHILOX:-0}" = 1 ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_philox.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_philox.txt 2>&1
rc=$?; tail -12 gpurun_out/pytest_philox.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
