#!/bin/bash
# Round 4, session 5: GELU on Linear2's A-load (bitwise tests, C2 end-to-end A/B), the RB default,
# then the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s5
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -k "agelu or defer_gelu or 224_rows or gemm" > $O/pt.log 2>&1; step pytest $?
tail -3 $O/pt.log
timeout -k 10 300 python tools/ab_toggle.py count_pipnet_amd.convnext_features.DEFER_GELU c2 --rounds 8 > $O/ab_c2_defer_gelu.log 2>&1; step abc2 $?
grep "^{" $O/ab_c2_defer_gelu.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; step bench $?
tail -1 $O/bench.log | cut -c1-600
LAB_ROUNDS=5 timeout -k 10 400 python tools/mlp_lab.py > $O/mlp_lab.log 2>&1; step mlplab $?
grep -v "^\[\|amdgpu.ids" $O/mlp_lab.log | tail -12
