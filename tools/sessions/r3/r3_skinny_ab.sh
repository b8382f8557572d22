#!/bin/bash
# skinny-M GEMM: tests, then C5 A/B (PIPNET_SKINNY=0/1) interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "skinny or splitk or linear" tests/test_gpu_c5.py "tests/test_gpu_parity.py::test_hip_forward_matches_reference_golden" > gpurun_out/r3_skinny_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r3_skinny_tests.log; grep -E "FAILED|^E  " gpurun_out/r3_skinny_tests.log | head
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for sk in 0 1; do
    PIPNET_SKINNY=$sk timeout -k 10 200 python tools/bench_configs.py --only c5,c5_bf16x3 --steps 30 --warmup 5 > gpurun_out/r3_skinny$sk.$r.log 2>&1 || exit $?
    echo "skinny=$sk run $r: $(grep '^{' gpurun_out/r3_skinny$sk.$r.log | python3 -c 'import sys,json
for l in sys.stdin: d=json.loads(l); print(d["config"], round(d["images_per_sec"]), round(d["ms_per_step"],4), end="  ")')"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_c5_skinny" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --only c5 --steps 13 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_c5_skinny.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"; head -12 $(find gpurun_out/prof_c5_skinny -name "*kernel_stats.csv") | cut -c1-160
