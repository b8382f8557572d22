#!/bin/bash
# Round 6: C2 end to end, product vs the wide-tile arm (variant 5 from 100 tiles, so the two-stream
# sub-batches of 23,328 rows take it too), default two-stream split, then one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ARMS="product wide" CFG=c2 ROUNDS=4 bash tools/sessions/r5_ab.sh || exit $?
cp gpurun_out/ab_c2.txt gpurun_out/ab_c2_wide_split2.txt
ARMS="product wide" CFG=c2 ROUNDS=3 EXTRA="--stream-split 1" bash tools/sessions/r5_ab.sh || exit $?
