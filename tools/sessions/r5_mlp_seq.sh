#!/bin/bash
# Round 5: sequential pixel-group passes (SEQ) of the fused CNBlock MLP vs the product shapes (tools/mlp_lab.hip
# 501-513), C5 and C2-half-batch shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
LAB_ROUNDS=5 LAB_SHAPES=96x65536,192x16384 LAB_VARIANTS='{"96": [0, 501, 502, 503, 504], "192": [4000, 511, 512, 513]}' \
  timeout -k 10 300 python tools/mlp_lab.py > gpurun_out/mlp_seq.txt 2>&1 || exit $?
LAB_ROUNDS=5 LAB_SHAPES=96x100352,192x25088,96x200704,192x50176 LAB_VARIANTS='{"96": [0, 501, 502, 503, 504], "192": [0, 511, 512, 513]}' \
  timeout -k 10 300 python tools/mlp_lab.py >> gpurun_out/mlp_seq.txt 2>&1 || exit $?
cat gpurun_out/mlp_seq.txt
