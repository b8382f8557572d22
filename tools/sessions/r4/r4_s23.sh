#!/bin/bash
# Round 4, session 23: eager vs HIP-graph replay per config (is the host's enqueue rate what
# limits the shorter forwards?)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s23
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python tools/bench_configs.py --only c2,c3,c5,c1 --graph --steps 20 --warmup 5 > $O/graph.log 2>&1; step graph $?
grep "^{" $O/graph.log | cut -c1-400
