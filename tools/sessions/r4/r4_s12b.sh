#!/bin/bash
# Round 4, sessions 12 + 13 in one call: fp32 GEMM plain vs non-temporal output stores (C2, C5)
# and the quad-layout bf16 head (test + C3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/sessions/r4_s13.sh || exit $?
bash tools/sessions/r4_s12.sh
