#!/bin/bash
# C5 bilinear split-K occupancy A/B (PIPNET_SPLITK_WG_PER_CU), interleaved, one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for w in 2 3 4 6; do
    PIPNET_SPLITK_WG_PER_CU=$w timeout -k 10 200 python tools/bench_configs.py --only c5 --steps 30 --warmup 5 > gpurun_out/r3_splitk$w.$r.log 2>&1 || exit $?
    echo "wg/cu=$w run $r: $(grep '^{' gpurun_out/r3_splitk$w.$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["images_per_sec"]), round(d["ms_per_step"],4))')"
  done
done
