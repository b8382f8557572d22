#!/bin/bash
# Round 6: C2 end to end, variant 4 everywhere (product) / fc1 only / off (tn4), with the default two-stream
# split and with one stream.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ARMS="product fc1only tn4" CFG=c2 ROUNDS=3 bash tools/sessions/r5_ab.sh || exit $?
cp gpurun_out/ab_c2.txt gpurun_out/ab_c2_split2.txt
ARMS="product fc1only tn4" CFG=c2 ROUNDS=3 EXTRA="--stream-split 1" bash tools/sessions/r5_ab.sh || exit $?
