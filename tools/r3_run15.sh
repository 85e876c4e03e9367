#!/bin/bash
# decode attention regressions (bf16 + fp8 cache), 13B fp8 decode timing, then a rocprof phase
# breakdown of one headline PPO step (Mistral-7B bf16, 256 rollouts).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r3
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "decode or fp8" > gpurun_out/r3/test_decode.log 2>&1 || { tail -40 gpurun_out/r3/test_decode.log; exit 1; }
tail -1 gpurun_out/r3/test_decode.log
timeout -k 10 300 python3 -u tools/decode_profile.py --model llama2-13b --fp8 --fp8-kv --batch 64 --prompt 320 --new 64 > gpurun_out/r3/dec13b_fp8kv_g1.log 2>&1 || { tail gpurun_out/r3/dec13b_fp8kv_g1.log; exit 1; }
grep "iter 2" gpurun_out/r3/dec13b_fp8kv_g1.log
GRIDS=gemm_big_kernel,gemm_small_kernel bash tools/ppo_phase_profile.sh || exit 1
grep -v "^[EW]2026" gpurun_out/prof_ppo/log.txt | tail -2 | cut -c1-300
head -5 gpurun_out/prof_ppo/phases.txt
