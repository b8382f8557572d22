#!/bin/bash
# Round 6: the one-segment-per-K-tile halo schedule (SEG = 1) against the product (SEG = 2), by ablation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
HALO_VARIANTS=${HALO_VARIANTS:-0,3000,3064,3128,3019,3083} timeout -k 10 300 python3 tools/halo_lab.py > gpurun_out/halo_lab.txt 2>&1
rc=$?; cat gpurun_out/halo_lab.txt; exit $rc
