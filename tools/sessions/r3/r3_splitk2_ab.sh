# C5 bilinear split-K slab depth / occupancy A/B after the weight fold (K = 2048), interleaved
mkdir -p gpurun_out
: > gpurun_out/splitk2_ab.txt
for run in 1 2; do
  for cfg in "256 2" "128 2" "128 4" "64 4" "64 8"; do
    set -- $cfg
    PIPNET_SPLITK_MIN_K=$1 PIPNET_SPLITK_WG_PER_CU=$2 timeout -k 10 120 python tools/bench_configs.py --only c5 --steps 30 > gpurun_out/sk.log 2>&1 || exit $?
    echo "min_k=$1 wg/cu=$2 run $run: $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/sk.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sk.log)" >> gpurun_out/splitk2_ab.txt
  done
done
cat gpurun_out/splitk2_ab.txt
