# bf16 epilogue cache-policy A/B across tiles: head / D (pp family) / E (D + generic + small-N halo), C3 interleaved
mkdir -p gpurun_out
: > gpurun_out/nt_ab3.log
for r in 1 2 3 4; do
  for v in head D E; do
    [ $v = head ] && f=libpipnet_amd_head.so || f=lib_$v.so
    PIPNET_AMD_LIB=$PWD/tools/ab_lib/$f PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 300 python tools/bench_configs.py --only c3 --steps 20 --warmup 5 > gpurun_out/nt_c3.log 2>&1 || exit $?
    echo "c3 $v run $r: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/nt_c3.log)" >> gpurun_out/nt_ab3.log
  done
done
cat gpurun_out/nt_ab3.log
