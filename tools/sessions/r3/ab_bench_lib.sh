# bench.py A/B: product library vs an A/B build ($AB_LIB), alternating, one box.
set -u
cd $GRAFT_REPO_ROOT
b() { timeout -k 10 300 python bench.py --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['value'],1), 'img/s', round(d['ms_per_step'],3), 'ms', 'dominant', round(d['roofline']['frac'],4))"; }
for i in 1 2; do
  b prod || exit 1
  PIPNET_AMD_LIB=$AB_LIB PIPNET_AMD_ALLOW_STALE=1 PIPNET_XCD_NG=0 b ab || exit 1
done
