#!/bin/bash
# Round 6: priority modes of the SEG 3 bf16 schedules: product (s_setprio around every M segment) vs prio0 (none)
# vs prio2 (one static s_setprio for the younger half), C3 interleaved + per layer.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ARMS="product prio0 prio2" CFG=c3 ROUNDS=${ROUNDS:-4} LAYERS=${LAYERS:-l3.c2,l4.c2,l3.c3,l4.c3,l3.c1,l4.c1} bash tools/sessions/r5_ab.sh
