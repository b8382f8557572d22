set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bf16.py -k "n64 or c3" > gpurun_out/pt_n64.log 2>&1; rc=$?; tail -5 gpurun_out/pt_n64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/conv_bf16_bench.py --batch 64 --only stem7x7,l1.c2 --tiles=-1,6,11 > gpurun_out/n64_bench.log 2>&1 || exit $?
cat gpurun_out/n64_bench.log
timeout -k 10 200 python tools/conv_bf16_bench.py --batch 128 --only l1.c2 --tiles=-1,6,11 >> gpurun_out/n64_bench.log 2>&1 || exit $?
tail -2 gpurun_out/n64_bench.log
