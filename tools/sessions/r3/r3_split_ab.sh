#!/bin/bash
# stream-split A/B on C2 / C5 / C3 (interleaved, one box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for n in 1 2 3; do
    timeout -k 10 300 python tools/bench_configs.py --only c2,c5,c3 --steps 20 --warmup 5 --stream-split $n > gpurun_out/r3_split$n.$r.log 2>&1 || exit $?
    echo "split=$n run $r"; grep "^{" gpurun_out/r3_split$n.$r.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(f\"  {d['config']:5s} {d['images_per_sec']:9.1f} img/s  {d['ms_per_step']:7.3f} ms  split {d['stream_split']}\")"
  done
done
