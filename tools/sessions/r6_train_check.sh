#!/bin/bash
# Round 6: the training parity tests after the per-step lr bookkeeping fix
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/train_check.txt 2>&1
rc=$?; grep -n "^E \|FAILED\|passed\|failed" gpurun_out/train_check.txt | tail -12; exit $rc
