#!/bin/bash
# Round 4 end-of-round evidence: GPU suite, smoke, default bench line, one-stream rocprof kernel
# stats (tools/final_evidence.sh).  PMC passes: tools/sessions/r4_pmc.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/final_evidence.sh
# lab: taller dwconv tiles with each weight row loaded once per workgroup (libdw_lab.so built
# with that form of convnext_dw.hpp)
DW_VARIANTS=0,7,40,41,42,43 DW_SHAPES=96x56,192x28,384x27,768x26,96x32,192x16 timeout -k 10 300 python tools/dw_lab.py > gpurun_out/dw_window.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/dw_window.log
