#!/bin/bash
# round-3 GPU session 2: ResNet training tests, GEMM clock stamps, steady-state copy count
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread "tests/test_gpu_train.py::test_suffix_training_matches_reference" -s > gpurun_out/r3_train.log 2>&1
rc=$?; echo "train rc $rc"; grep -E "PASSED|FAILED|running statistics|Error" gpurun_out/r3_train.log | tail -20
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/gemm_stamps.py s384_fc1,s768_fc1,s768_fc2,s384_fc2 > gpurun_out/r3_stamps.log 2>&1 || exit $?
grep -v "amdgpu.ids" gpurun_out/r3_stamps.log
for cfg in c3 c5; do
  for st in 3 13; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_copy_${cfg}_$st" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --only $cfg --steps $st --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_copy_${cfg}_$st.log" 2>&1) || exit $?
    f=$(find gpurun_out/prof_copy_${cfg}_$st -name "*kernel_stats.csv" | head -1)
    echo "$cfg steps=$st: $(grep -c . $f) kernels; copies: $(grep -E 'copyBuffer|fillBuffer' $f | cut -d, -f1,2 | tr '\n' ' ')"
  done
done
