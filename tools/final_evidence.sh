#!/bin/bash
# End-of-round evidence on one GPU box: full GPU suite, smoke, the default bench line (with the
# CPU baseline), and a rocprofv3 kernel-stats run of the same bench with ONE stream
# (--stream-split 1): every launch in the kept CSV is then a full-batch launch, so its per-kernel
# averages are the ones bench.py's roofline pass times with HIP events (two concurrent half-batch
# launches each take about as long as a full one and would halve the apparent rate).
# Outputs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_final.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu_final.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.txt 2>&1 || exit $?
tail -1 gpurun_out/smoke_final.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_final.log | cut -c1-300
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_final" -o run \
  --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --stream-split 1 > "$R/gpurun_out/prof_final.log" 2>&1) || exit $?
echo "final evidence done"
