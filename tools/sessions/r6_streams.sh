#!/bin/bash
# Round 6: C2 / C5 sub-batch stream splits after the wide fp32 tile (tools/ab_toggle.py streams:1:2:3:4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/streams.txt
: > $out
for c in ${CFGS:-c2}; do
  timeout -k 10 500 python tools/ab_toggle.py ${ARMS:-streams:1:2:3:4} $c --rounds 4 > gpurun_out/streams_$c.log 2>&1
  rc=$?; grep '^{' gpurun_out/streams_$c.log | cut -c1-220 >> $out; [ $rc -eq 0 ] || { tail -5 gpurun_out/streams_$c.log; exit $rc; }
done
cat $out
