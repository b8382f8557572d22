#!/bin/bash
# Round 5: raster group budgets of the bf16 (C3) and fp32 (C2) GEMM families, built as separate
# libraries (tools/ab_build.py): end-to-end A/B in interleaved rounds of separate processes, then one
# rocprofv3 FETCH_SIZE pass of bench.py per fp32 arm (HBM/MALL read bytes per kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
mkdir -p gpurun_out
out=gpurun_out/ab_raster.txt
: > $out
lib_of() { if [ $1 = product ]; then echo $R/count_pipnet_amd/libpipnet_amd.so; else echo $R/tools/ab/libpipnet_$1.so; fi; }
for r in 1 2 3; do
  for v in product g05m g025m g1; do
    PIPNET_AMD_LIB=$(lib_of $v) timeout -k 10 180 python tools/bench_configs.py --only c3 --steps 20 > gpurun_out/ab_c3_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c3 arm $v failed rc=$rc" >> $out; exit $rc; }
    echo "c3 round $r $v $(grep '^{' gpurun_out/ab_c3_$v.log | head -1 | cut -c1-110)" >> $out
  done
  for v in product gf1m gf1; do
    PIPNET_AMD_LIB=$(lib_of $v) timeout -k 10 180 python tools/bench_configs.py --only c2 --steps 20 > gpurun_out/ab_c2_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "c2 arm $v failed rc=$rc" >> $out; exit $rc; }
    echo "c2 round $r $v $(grep '^{' gpurun_out/ab_c2_$v.log | head -1 | cut -c1-110)" >> $out
  done
done
export TMPDIR=/tmp
for v in product gf1m gf1; do
  (cd /tmp && PIPNET_AMD_LIB=$(lib_of $v) timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$R/gpurun_out/fetch_$v" -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --stream-split 1 > "$R/gpurun_out/fetch_$v.log" 2>&1)
  rc=$?; echo "[fetch $v] exit $rc" >> $out; [ $rc -eq 0 ] || exit $rc
done
cat $out
