# persistent-tile non-temporal epilogue A/B: its GPU tests, then 1x1 layers head vs this tree, then C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py -k "persistent or dual or c3" > gpurun_out/pt_nt.log 2>&1; rc=$?; tail -2 gpurun_out/pt_nt.log; [ $rc -eq 0 ] || exit $rc
L="l2.c3,l3.c1,l3.c3,l4.c1,l4.c3,l4.ds"
PIPNET_AMD_LIB=$PWD/tools/ab_lib/libpipnet_amd_head.so PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 200 python tools/conv_bf16_bench.py --batch 64 --only $L --tiles=-1 > gpurun_out/nt_ab.log 2>&1 || exit $?
echo "--- nt epilogue" >> gpurun_out/nt_ab.log
timeout -k 10 200 python tools/conv_bf16_bench.py --batch 64 --only $L --tiles=-1 >> gpurun_out/nt_ab.log 2>&1 || exit $?
for r in 1 2; do
PIPNET_AMD_LIB=$PWD/tools/ab_lib/libpipnet_amd_head.so PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 300 python tools/bench_configs.py --only c3 --steps 20 --warmup 5 > gpurun_out/nt_c3_old.log 2>&1 || exit $?
echo "old: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/nt_c3_old.log)" >> gpurun_out/nt_ab.log
timeout -k 10 300 python tools/bench_configs.py --only c3 --steps 20 --warmup 5 > gpurun_out/nt_c3_new.log 2>&1 || exit $?
echo "new: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/nt_c3_new.log)" >> gpurun_out/nt_ab.log
done
grep -v amdgpu.ids gpurun_out/nt_ab.log
