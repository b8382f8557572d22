# head kernels' proto-map stores non-temporal: head vs this tree, C3 / C5 / C2 interleaved
mkdir -p gpurun_out
: > gpurun_out/nt_head_ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_c5.py tests/test_gpu_parity.py > gpurun_out/pt_nt_head.log 2>&1 || { tail -5 gpurun_out/pt_nt_head.log; exit 1; }
tail -1 gpurun_out/pt_nt_head.log >> gpurun_out/nt_head_ab.log
for r in 1 2 3; do
  for v in head new; do
    if [ $v = head ]; then E="PIPNET_AMD_LIB=$PWD/tools/ab_lib/libpipnet_amd_head.so PIPNET_AMD_ALLOW_STALE=1"; else E=""; fi
    env $E timeout -k 10 300 python tools/bench_configs.py --only c3,c5 --steps 20 --warmup 5 > gpurun_out/nth.log 2>&1 || exit $?
    echo "$v run $r: $(grep -o '"config": "c[0-9]", "images_per_sec": [0-9.]*' gpurun_out/nth.log | tr '\n' ' ')" >> gpurun_out/nt_head_ab.log
  done
done
cat gpurun_out/nt_head_ab.log
