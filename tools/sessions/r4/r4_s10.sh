#!/bin/bash
# Round 4, session 10: running row pointers in the bf16 pp-family and fp32 GEMM epilogues (no per-store
# multiplies): GPU bf16 tests, per-layer timing, C3 end to end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/r4s10
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$1] exit $2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1; step pytest $?
tail -1 $O/pt.log
timeout -k 10 300 python tools/c3_diag.py --tiles 9,5 --reps 20 --only l3.c1,l4.c1,l3.c3,l4.ds,l4.c3 > $O/c3_diag.log 2>&1; step c3diag $?
grep -v "amdgpu.ids" $O/c3_diag.log
timeout -k 10 400 python tools/ab_toggle.py streams:2:1 c3 --rounds 5 > $O/c3_streams.txt 2>&1; step c3 $?
grep "^{" $O/c3_streams.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; step bench $?
python - "$O/bench.log" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", round(r["value"]), "ms", round(r["ms_per_step"], 3), "dominant frac", round(r["roofline"]["frac"], 3))
for k, v in r.get("extra", {}).items():
    print(k, round(v["value"]), "ms", round(v["ms_per_step"], 3), "frac", round(v["roofline"]["frac"], 3))
PY
