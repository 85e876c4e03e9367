#!/bin/bash
# fp8 K/V cache: kernel numerics, decode/generation regressions, then the 13B batch-64 decode step.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r3
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8kv or kv_store_fp8" > gpurun_out/r3/test_fp8kv.log 2>&1 || { tail -40 gpurun_out/r3/test_fp8kv.log; exit 1; }
tail -3 gpurun_out/r3/test_fp8kv.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py tests/test_pipeline_gpu.py \
  > gpurun_out/r3/test_models.log 2>&1 || { tail -40 gpurun_out/r3/test_models.log; exit 1; }
tail -2 gpurun_out/r3/test_models.log
timeout -k 10 300 python3 -u tools/decode_profile.py --model llama2-13b --fp8 --batch 64 --prompt 320 --new 64 > gpurun_out/r3/dec13b_bf16kv.log 2>&1 || { tail gpurun_out/r3/dec13b_bf16kv.log; exit 1; }
grep iter gpurun_out/r3/dec13b_bf16kv.log
timeout -k 10 300 python3 -u tools/decode_profile.py --model llama2-13b --fp8 --fp8-kv --batch 64 --prompt 320 --new 64 > gpurun_out/r3/dec13b_fp8kv.log 2>&1 || { tail gpurun_out/r3/dec13b_fp8kv.log; exit 1; }
grep iter gpurun_out/r3/dec13b_fp8kv.log
