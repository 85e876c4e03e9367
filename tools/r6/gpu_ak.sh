#!/bin/bash
# Round-6 call AK: 4-rank data-parallel rehearsal of bench.py on one GPU over gloo (launcher, rank
# setup, GradSync, metric reduction at world 4; not a scaling point)
set -o pipefail
mkdir -p gpurun_out/ak
RAGTL_DIST_BACKEND=gloo timeout -k 10 1000 python -u bench.py --gpus 4 --steps 2 --warmup 1 --skip-latency --rollout-batch 32 --model tiny-mistral --encoder tiny-bert --reward-encoder same > gpurun_out/ak/dp4_gloo.log 2>&1 || exit 1
tail -1 gpurun_out/ak/dp4_gloo.log | cut -c1-600
