#!/bin/bash
# Round 4 end-of-round evidence: GPU suite, smoke, default bench line, one-stream rocprof kernel
# stats (tools/final_evidence.sh).  PMC passes: tools/sessions/r4_pmc.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/final_evidence.sh
