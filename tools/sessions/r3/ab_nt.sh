# A/B of the fp32 GEMM raster / store policy (lab builds tools/lib_xcdng.so, lib_ntstore.so):
# (The XCD-slab raster and PIPNET_GEMM_NT_STORE switches exist at commit "fp32 GEMM lab switches"; NT stores
# became the product default and the slab raster was removed in the commit after it.)
# output digests (must match), gemm_bench timings, FETCH_SIZE per shape.
set -u
cd $GRAFT_REPO_ROOT
X=$PWD/tools/lib_xcdng.so; N=$PWD/tools/lib_ntstore.so
run() { timeout -k 10 200 "$@"; }
cfg() {  # $1 tag, $2 lib ('' = product), $3 NG
  local tag=$1
  if [ -n "$2" ]; then export PIPNET_AMD_LIB=$2 PIPNET_AMD_ALLOW_STALE=1; else unset PIPNET_AMD_LIB PIPNET_AMD_ALLOW_STALE; fi
  export PIPNET_XCD_NG=$3
  echo "== $tag" && run python tools/ab_digest.py 2>&1 | grep digest &&
  run python tools/gemm_bench.py > gpurun_out/ab_$tag.log 2>&1 && grep -E "s384|s768|network" gpurun_out/ab_$tag.log | grep -v '^\[' &&
  PMC_OUT=pmc_$tag PMC_SETS="FETCH_SIZE" PMC_CMD="tools/gemm_bench.py --iters 3" run bash tools/pmc_generic.sh > gpurun_out/pmc_$tag.log 2>&1
}
cfg prod "" 0 && cfg ng1 $X 1 && cfg ng2 $X 2 && cfg ng4 $X 4 && cfg ng8 $X 8 && cfg nt_ng0 $N 0 && cfg nt_ng2 $N 2 && cfg prod2 "" 0
