#!/bin/bash
# Round 4, session 18: round-4 bf16 conv tile rule (tile 12, short-K conv3 + identity off the
# ping-pong tiles): GPU tests, C3 A/B against round 3's rule, per-layer timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s18
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_capi_symbols.py -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 400 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_tile_rule:0:1 c3 --rounds 7 > $O/ab_c3_rule.txt 2>&1; step abc3 $?
grep "^{" $O/ab_c3_rule.txt
timeout -k 10 300 python tools/conv_bf16_bench.py --batch 64 --tiles=-1 --reps 20 > $O/conv_auto.log 2>&1; step bench $?
grep -v amdgpu.ids $O/conv_auto.log
