#!/bin/bash
# Round 6: ablation of the product dwconv7 + LayerNorm kernel (tools/dw_lab.py --abl6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared tools/dw_lab.hip -o tools/libdw_lab.so -I include 2>/dev/null || exit 1
DW_SHAPES=384x27 DW_VARIANTS=0 timeout -k 10 300 python3 tools/dw_lab.py --abl6 > gpurun_out/dw_abl.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/dw_abl.txt; exit $rc
