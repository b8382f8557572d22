# vectorised fp32 softmax-pool head: its GPU tests + the C2 parity tests, then C2 head-lib vs this tree, interleaved
mkdir -p gpurun_out
: > gpurun_out/spf32_ab.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_parity.py > gpurun_out/pt_spf32.log 2>&1 || { tail -5 gpurun_out/pt_spf32.log; exit 1; }
tail -1 gpurun_out/pt_spf32.log >> gpurun_out/spf32_ab.log
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then E="PIPNET_AMD_LIB=$PWD/tools/ab_lib/libpipnet_amd_head.so PIPNET_AMD_ALLOW_STALE=1"; else E=""; fi
    env $E timeout -k 10 300 python tools/bench_configs.py --only c2 --steps 20 --warmup 5 > gpurun_out/spf.log 2>&1 || exit $?
    echo "$v run $r: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/spf.log)" >> gpurun_out/spf32_ab.log
  done
done
cat gpurun_out/spf32_ab.log
