#!/bin/bash
# round 5, GPU call AV: batch-1 RAG answer loop kernel stats on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5av
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb1 -o run -- python3 -u bench.py --steps 0 --latency-queries 16 > $O/log.txt 2>&1 || { tail -20 $O/log.txt; exit 1; }
find /tmp/profb1 -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
grep "p50" $O/log.txt | head -2 | cut -c1-200
