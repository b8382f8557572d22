#!/bin/bash
# Round 6: the fp32 GEMM on v_mfma_f32_16x16x4_f32 (lab variants 40 / 41 / 42 = product tiles 0 / 1 / 2 with
# the 16x16x4 MFMA) against the product 32x32x2 forms on C2's shapes (the vendor fp32 GEMM uses 16x16x4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/gemm_lab.hip -o tools/libgemm_lab.so -I include 2>/dev/null || exit 1
LAB_VARIANTS=${LAB_VARIANTS:-0,2,40,42} LAB_GROUPS=${LAB_GROUPS:-8} timeout -k 10 400 python3 tools/gemm_lab.py > gpurun_out/gemm16.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/gemm16.txt; exit $rc
