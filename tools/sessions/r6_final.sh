#!/bin/bash
# Round 6 evidence on one GPU box: PMC passes (clock / MFMA busy, FETCH_SIZE, WRITE_SIZE; separate runs, one stream)
# over C2 (bench.py), C3 and C5 (tools/bench_configs.py), rows keyed by the FULL kernel name (tools/pmc_summary.py); the
# traffic files installed under profiles/ (bench.py's roofline.traffic reads them, digest-checked); then
# tools/final_evidence.sh (GPU suite, smoke, the default bench line with the CPU baseline, rocprofv3 kernel stats of the
# bench with --stream-split 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_PMC:-0}" != 1 ]; then
  bash tools/pmc_all.sh || exit $?
  python3 - <<'PY' || exit $?
import json, shutil
shutil.copy("gpurun_out/pmc/traffic_latest.json", "profiles/traffic_latest.json")
merged = {}
for d in ("pmc", "pmc_c3", "pmc_c5"):
    merged.update(json.load(open(f"gpurun_out/{d}/traffic_kernels.json")))
json.dump(merged, open("profiles/traffic_kernels.json", "w"), indent=1)
print("traffic installed:", len(merged), "kernels")
PY
fi
bash tools/final_evidence.sh || exit $?
echo "r6 final done"
