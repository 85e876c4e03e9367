#!/bin/bash
# fp8 training forward (config 5): parity + kernel tests, then the 13B pipeline with and without it.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py \
  -k "fp8 or swiglu or lora" > gpurun_out/r3/test_fp8train.log 2>&1 || { tail -40 gpurun_out/r3/test_fp8train.log; exit 1; }
tail -1 gpurun_out/r3/test_fp8train.log
for ft in fp8-train no-fp8-train; do
  timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 --$ft > gpurun_out/r3/bench_pipeline_$ft.log 2>&1 || { tail -20 gpurun_out/r3/bench_pipeline_$ft.log; exit 1; }
  echo "== $ft"; grep -v "^[EW]2026" gpurun_out/r3/bench_pipeline_$ft.log | tail -1 | cut -c1-160
  grep -o '"ppo_phase_s_per_step.*' gpurun_out/r3/bench_pipeline_$ft.log
  grep "warmup\|step " gpurun_out/r3/bench_pipeline_$ft.log | tail -3
done
