#!/bin/bash
# qkv NT planner A/B (all-256 tiles vs 32 row tiles at 256 + 6 at 128) and a 10-step headline bench
set -o pipefail
mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
for c in 0.55 0.45; do
  RT_GEMM_BN128_COST=$c timeout -k 10 200 python3 -u tools/gemm_big_probe.py --M 9632 7000 12000 --shapes qkv,o,down --cases nt,nn,lib_nt --rounds 3 > gpurun_out/r3/planner_cost_$c.log 2>&1 || exit 1
  echo "cost $c"; cat gpurun_out/r3/planner_cost_$c.log | grep M=
done
timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 1 > gpurun_out/r3/bench_final_10steps.log 2>&1 || { tail -20 gpurun_out/r3/bench_final_10steps.log; exit 1; }
tail -1 gpurun_out/r3/bench_final_10steps.log
