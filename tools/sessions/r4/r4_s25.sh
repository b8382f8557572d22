#!/bin/bash
# Round 4, session 25: CountPIPNet sub-batch split with the interleaved enqueue (C5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s25
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest_graph.txt 2>&1; step graph $?
tail -3 $O/pytest_graph.txt
timeout -k 10 400 python tools/ab_toggle.py streams:1:2:3 c5 --rounds 6 > $O/ab_c5_streams.txt 2>&1; step streams $?
grep "^{\|bitwise" $O/ab_c5_streams.txt
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.INTERLEAVE c5 --stream-split 2 --rounds 6 > $O/ab_c5_interleave.txt 2>&1; step interleave $?
grep "^{\|bitwise" $O/ab_c5_interleave.txt
