#!/bin/bash
# W8A8 on the gemm_big schedule: numerics, A/B vs the 256x256 fp8 kernel, 13B pipeline bench.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8 or swiglu" > gpurun_out/r3/test_w8a8.log 2>&1 || { tail -40 gpurun_out/r3/test_w8a8.log; exit 1; }
tail -1 gpurun_out/r3/test_w8a8.log
timeout -k 10 300 python3 -u tools/fp8_w8a8_probe.py > gpurun_out/r3/w8a8_big.log 2>&1 || { tail gpurun_out/r3/w8a8_big.log; exit 1; }
RT_GEMM_FP8_256=1 timeout -k 10 300 python3 -u tools/fp8_w8a8_probe.py > gpurun_out/r3/w8a8_256.log 2>&1 || { tail gpurun_out/r3/w8a8_256.log; exit 1; }
grep -h '"M": 20480' gpurun_out/r3/w8a8_big.log gpurun_out/r3/w8a8_256.log | cut -c1-200
timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline5.log 2>&1 || { tail -20 gpurun_out/r3/bench_pipeline5.log; exit 1; }
grep -v "^[EW]2026" gpurun_out/r3/bench_pipeline5.log | tail -1 | cut -c1-200
grep -o '"ppo_phase_s_per_step.*' gpurun_out/r3/bench_pipeline5.log
