#!/bin/bash
# Round 4, session 19: which half of the round-4 tile rule costs C3 end to end?  modes 0 = round
# 3, 1 = conv3 + identity K <= 256 off the ping-pong tiles only, 2 = tile 12 for tile 4 only, 3 = both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s19
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_tile_rule:0:1:2:3 c3 --rounds 7 > $O/ab_c3_rule.txt 2>&1; step abc3 $?
grep "^{" $O/ab_c3_rule.txt
timeout -k 10 600 python tools/ab_toggle.py fn:count_pipnet_amd.kernels.conv_bf16_tile_rule:0:1:2:3 c3 --rounds 5 --stream-split 1 > $O/ab_c3_rule_s1.txt 2>&1; step abc3s1 $?
grep "^{" $O/ab_c3_rule_s1.txt
