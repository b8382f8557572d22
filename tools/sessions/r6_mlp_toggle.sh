#!/bin/bash
# Round 6: C2 with the fused narrow-stage MLP off / on (tools/ab_toggle.py, interleaved in one process)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.convnext_features.FUSED_MLP c2 --rounds 5 > gpurun_out/mlp_toggle.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/mlp_toggle.log | tail -12; exit $rc
