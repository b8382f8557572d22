# persistent-tile epilogue cache-policy A/B: head / ntall / B (nt stores without residual) / C (nt identity loads only)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/nt_ab2.log
L="l2.c3,l3.c1,l3.c3,l4.c1,l4.c3,l4.ds"
for v in head ntall B C; do
  [ $v = head ] && f=libpipnet_amd_head.so || f=lib_$v.so
  echo "--- $v" >> gpurun_out/nt_ab2.log
  PIPNET_AMD_LIB=$PWD/tools/ab_lib/$f PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 200 python tools/conv_bf16_bench.py --batch 64 --only $L --tiles=-1 2>&1 | grep -v amdgpu.ids >> gpurun_out/nt_ab2.log || exit $?
done
for r in 1 2 3; do
  for v in head ntall B C; do
    [ $v = head ] && f=libpipnet_amd_head.so || f=lib_$v.so
    PIPNET_AMD_LIB=$PWD/tools/ab_lib/$f PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 300 python tools/bench_configs.py --only c3 --steps 20 --warmup 5 > gpurun_out/nt_c3.log 2>&1 || exit $?
    echo "c3 $v run $r: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/nt_c3.log)" >> gpurun_out/nt_ab2.log
  done
done
cat gpurun_out/nt_ab2.log
