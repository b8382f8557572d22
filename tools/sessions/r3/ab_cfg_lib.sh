# bench_configs.py A/B: product library vs an A/B build ($AB_LIB), alternating, one box.
# AB_CFGS = space-separated config names (tools/bench_configs.py --only).
set -u
cd $GRAFT_REPO_ROOT
for c in ${AB_CFGS}; do
  for i in 1 2; do
    timeout -k 10 200 python tools/bench_configs.py --only $c --steps ${AB_STEPS:-5} 2>/dev/null | grep "^{" | cut -c1-120 | sed 's/^/prod /' || exit 1
    PIPNET_AMD_LIB=$AB_LIB PIPNET_AMD_ALLOW_STALE=1 timeout -k 10 200 python tools/bench_configs.py --only $c --steps ${AB_STEPS:-5} 2>/dev/null | grep "^{" | cut -c1-120 | sed 's/^/ab   /' || exit 1
  done
done
