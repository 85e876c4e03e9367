#!/bin/bash
# Round-6 call AP: no fused-layer image refresh for big-batch decodes — GPU tier, bench
set -o pipefail
mkdir -p gpurun_out/ap
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ap/gputests.log 2>&1
rc=$?; tail -2 gpurun_out/ap/gputests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/ap/bench_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"p50_rag_latency_s": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/ap/bench_$i.log
done
