# fused stem + max-pool check: bf16 + capi GPU tests, C3 parity tests, C3 in-process A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py tests/test_capi_symbols.py tests/test_gpu_parity.py > gpurun_out/pt_stem_pool.log 2>&1; rc=$?; tail -3 gpurun_out/pt_stem_pool.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.resnet_hip.STEM_POOL c3 --rounds 7 > gpurun_out/ab_stem_pool_c3.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_stem_pool_c3.txt
