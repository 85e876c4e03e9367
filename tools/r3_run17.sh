#!/bin/bash
# Config 5 end to end with the fp8 K/V cache: pipeline bench + rocprof phase breakdown of the 13B
# PPO step, then fp8 decode table (dispatch now picks bf16 where fp8 was slower).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline13b_fp8kv.log 2>&1 || { tail -20 gpurun_out/r3/bench_pipeline13b_fp8kv.log; exit 1; }
grep -v "^[EW]2026" gpurun_out/r3/bench_pipeline13b_fp8kv.log | tail -2 | cut -c1-600
timeout -k 10 700 bash tools/prof_pipeline13b.sh || exit 1
head -30 gpurun_out/prof13b/phases.txt | grep -A12 "== rollout"
