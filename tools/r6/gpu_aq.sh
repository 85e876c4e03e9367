#!/bin/bash
# Round-6 call AQ: same-box A/B of the decode-image refresh gating (REFRESH_ONLY_USED 1 / 0), with
# the batch-1 latency bench first (it creates the images a PPO rollout used to refresh every step)
set -o pipefail
mkdir -p gpurun_out/aq
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 600 python -u tools/r6/bench_with.py rag_tl_domainllm_optimizer_amd.models.decoder.REFRESH_ONLY_USED=$v -- --steps 3 --warmup 1 > gpurun_out/aq/b_${v}_$i.log 2>&1 || exit 1
    echo "refresh_only_used=$v $(grep -o '"value": [0-9.]*' gpurun_out/aq/b_${v}_$i.log) $(grep -o '"time/rollout": [0-9.]*' gpurun_out/aq/b_${v}_$i.log)"
  done
done
