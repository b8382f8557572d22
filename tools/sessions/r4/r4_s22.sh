#!/bin/bash
# Round 4, session 22: sub-batch forwards enqueued block by block (pipnet.INTERLEAVE) + the
# cache-miss stream sync: GPU tests, then C2 / C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s22
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.INTERLEAVE c2 --rounds 7 > $O/ab_c2.txt 2>&1; step c2 $?
grep "^{" $O/ab_c2.txt
timeout -k 10 400 python tools/ab_toggle.py count_pipnet_amd.pipnet.INTERLEAVE c3 --rounds 7 > $O/ab_c3.txt 2>&1; step c3 $?
grep "^{" $O/ab_c3.txt
