#!/bin/bash
# Round-6 call AO: same-box A/B of the LoRA slab split plans (round-6 sweep vs round-5 plans)
set -o pipefail
mkdir -p gpurun_out/ao
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 600 python -u tools/r6/bench_with.py rag_tl_domainllm_optimizer_amd.ops.linear.SLAB_SPLITS_R6=$v -- --steps 3 --warmup 1 --skip-latency > gpurun_out/ao/b_${v}_$i.log 2>&1 || exit 1
    echo "splits_r6=$v $(grep -o '"value": [0-9.]*' gpurun_out/ao/b_${v}_$i.log) $(grep -o '"time/update": [0-9.]*' gpurun_out/ao/b_${v}_$i.log)"
  done
done
