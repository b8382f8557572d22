#!/bin/bash
# round-3 (late) check on a GPU box: the GPU tests of the touched paths, then one bench line
# summarised (C2 value, C3 / C5 img/s).  TESTS overrides the pytest selection.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_c5.py tests/test_gpu_parity.py tests/test_gpu_graph.py}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $T \
  > gpurun_out/pytest_check.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_check.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_check.log 2>&1 || exit $?
tail -1 gpurun_out/bench_check.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
e = d.get('extra', {})
print('C2', round(d['value'], 1), 'frac', round(d['roofline']['frac'], 4),
      '| C3', round(e.get('c3', {}).get('value', 0), 1), '| C5', round(e.get('c5', {}).get('value', 0), 1),
      round(e.get('c5', {}).get('ms_per_step', 0), 4), 'ms')"
