#!/bin/bash
# round 5, GPU call AE: deferred attention-partition merge into the o-projection GEMV — tests, latency A/B, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "deferred_merge or test_decode_step_fused" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for dm in on off; do
    echo "== defer-merge $dm" >> $O/lat.log
    timeout -k 10 300 python -u bench.py --steps 0 --latency-queries 24 --defer-merge $dm >> $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
  done
done
grep -E "==|p50=" $O/lat.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profd -o run -- python3 -u bench.py --steps 0 --latency-queries 8 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find /tmp/profd -name "*kernel_stats.csv" -exec cp {} $O/defer_on_kernel_stats.csv \;
