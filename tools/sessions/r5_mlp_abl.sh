#!/bin/bash
# Round 5: time breakdown of the fused CNBlock MLP by ablation (tools/mlp_lab.hip 1000 * shape + ABL bits):
# C5 shapes (stage 1 96 x 65,536 px, stage 2 192 x 16,384) and C2's two-stream half batches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
B="0 1 2 4 8 16 3 12 18"
j() { local base=$1; local out=""; for b in $B; do out="$out$((base + b)),"; done; echo "[${out%,}]"; }
LAB_ROUNDS=3 LAB_SHAPES=96x65536,192x16384 LAB_VARIANTS="{\"96\": $(j 3000), \"192\": $(j 4000)}" \
  timeout -k 10 300 python tools/mlp_lab.py > gpurun_out/mlp_abl.txt 2>&1 || exit $?
LAB_ROUNDS=3 LAB_SHAPES=96x100352,192x25088 LAB_VARIANTS="{\"96\": $(j 1000), \"192\": $(j 2000)}" \
  timeout -k 10 300 python tools/mlp_lab.py >> gpurun_out/mlp_abl.txt 2>&1 || exit $?
cat gpurun_out/mlp_abl.txt
