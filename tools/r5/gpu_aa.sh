#!/bin/bash
# round 5, GPU call AA: decode-attention weight prefetch — bitwise test, batch-1 latency A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "prefetch_workgroups or test_decode_step_fused" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for pf in 1 0; do
    echo "== attn_prefetch=$pf" >> $O/lat.log
    timeout -k 10 300 python -u bench.py --steps 0 --latency-queries 24 --tuning attn_prefetch=$pf >> $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
  done
done
grep -E "==|p50" $O/lat.log
