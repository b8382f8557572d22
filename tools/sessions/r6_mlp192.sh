#!/bin/bash
# Round 6: C2 stage 2 (C = 192, 28 x 28) fused MLP vs the two GEMMs (MLP192_FUSED_MAX_PIXELS 2^30 / 512)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_toggle.py attr:count_pipnet_amd.convnext_features.MLP192_FUSED_MAX_PIXELS:1073741824:512 c2 \
  --rounds 5 > gpurun_out/mlp192.log 2>&1
rc=$?; grep '^{' gpurun_out/mlp192.log | cut -c1-250; [ $rc -eq 0 ] || tail -5 gpurun_out/mlp192.log; exit $rc
