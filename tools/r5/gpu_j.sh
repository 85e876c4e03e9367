#!/bin/bash
# round 5, GPU call J: sampler window path (bitwise vs the full-row search) + batch-1 latency
# A/B (sample_window 1 vs 0) and a kernel-trace of the answer loop
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k sampler --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for w in 1 0; do
  timeout -k 10 400 python -u bench.py --steps 0 --latency-queries 16 --tuning sample_window=$w > $O/lat_w$w.log 2>&1 || { tail -20 $O/lat_w$w.log; exit 2; }
  tail -1 $O/lat_w$w.log | cut -c1-400
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o b1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 0 --latency-queries 8 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 3; }
grep -i "sample\|attn_decode" $GRAFT_REPO_ROOT/$O/prof/b1_kernel_stats.csv | cut -c1-200
