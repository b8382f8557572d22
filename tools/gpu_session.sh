#!/bin/bash
# One GPU-box session: gpu tests -> smoke -> bench -> rocprof kernel summary.
# Test failures (exit 1) do not stop the session; faults, aborts and time limits do.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit code, $2 = step name
  local rc=$1
  echo "[$2] exit $rc" | tee -a gpurun_out/session.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "fatal exit in $2; stopping" | tee -a gpurun_out/session.log; exit "$rc"; fi
}
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; stop_if_fatal $? tests; tail -30 gpurun_out/pytest_gpu.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1; stop_if_fatal $? smoke; tail -3 gpurun_out/smoke.log ;;
    lab)   timeout -k 10 600 python tools/gemm_lab.py > gpurun_out/gemm_lab.log 2>&1; stop_if_fatal $? lab; grep -v "^\[\|amdgpu.ids" gpurun_out/gemm_lab.log | tail -20 ;;
    dwlab) timeout -k 10 300 python tools/dw_lab.py > gpurun_out/dw_lab.log 2>&1; stop_if_fatal $? dwlab; grep -v "^\[\|amdgpu.ids" gpurun_out/dw_lab.log | tail -8 ;;
    cfgs)  timeout -k 10 600 python tools/bench_configs.py > gpurun_out/bench_configs.log 2>&1; stop_if_fatal $? cfgs; grep "^{" gpurun_out/bench_configs.log ;;
    convbf) timeout -k 10 300 python tools/conv_bf16_bench.py > gpurun_out/conv_bf16.log 2>&1; stop_if_fatal $? convbf; grep -v "^\[" gpurun_out/conv_bf16.log | tail -20 ;;
    profcfg) (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${CFG}" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --only ${CFG} --steps 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_${CFG}.log" 2>&1); stop_if_fatal $? profcfg ;;
    pmcg)  timeout -k 10 900 bash tools/pmc_generic.sh > gpurun_out/pmcg.log 2>&1; stop_if_fatal $? pmcg; tail -60 gpurun_out/pmcg.log ;;
    gemm)  timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; stop_if_fatal $? gemm; grep -v "^\[" gpurun_out/gemm_bench.log | tail -20 ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; stop_if_fatal $? bench; tail -3 gpurun_out/bench.log ;;
    prof)  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1); stop_if_fatal $? prof; find gpurun_out/prof -name "*stats*" | head ;;
    pmc)   timeout -k 10 900 bash tools/pmc.sh > gpurun_out/pmc.log 2>&1; stop_if_fatal $? pmc; tail -25 gpurun_out/pmc.log ;;
    fold)  timeout -k 10 180 python tools/fold_bench.py > gpurun_out/fold_bench.txt 2>&1; stop_if_fatal $? fold; tail -1 gpurun_out/fold_bench.txt ;;
    bf16lab) LAB_ABL=${LAB_ABL:-0,2,32,34,-1} LAB_SHAPES=${LAB_SHAPES:-sq4096,sq8192,l3c1,l4c1,l4ds,l3c3} timeout -k 10 600 python tools/bf16_lab.py > gpurun_out/bf16_lab.log 2>&1; stop_if_fatal $? bf16lab; grep -v "^\[\|amdgpu.ids" gpurun_out/bf16_lab.log | tail -20 ;;
  esac
done
exit 0
