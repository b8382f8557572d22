# tile 11 (small-N LDS-halo 3x3) check: its GPU tests, per-layer timings vs the generic tiles, C3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py > gpurun_out/pt_n64.log 2>&1; rc=$?; tail -3 gpurun_out/pt_n64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/conv_bf16_bench.py --batch 64 --only l1.c2,l2.c2 --tiles=-1,0,4,6,11 > gpurun_out/n64_bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/n64_bench.log
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.kernels.CONV3X3_N64_HALO c3 --rounds 7 > gpurun_out/ab_n64_c3.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_n64_c3.txt
