#!/bin/bash
# round 5, GPU call AF: deferred merge with fewer, longer partitions (records read by every o-GEMV workgroup)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5af
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for dm in off 128 256 on; do
    echo "== defer-merge $dm" >> $O/lat.log
    timeout -k 10 300 python -u bench.py --steps 0 --latency-queries 24 --defer-merge $dm >> $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
  done
done
grep -E "==|p50=" $O/lat.log
