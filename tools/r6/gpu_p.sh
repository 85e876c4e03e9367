#!/bin/bash
# Round-6 call P: fixed-order slab LoRA backward (dU, dA, dB) — targeted tests, reproducibility test, bench
set -o pipefail
mkdir -p gpurun_out/p
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_zz_dist_gpu.py tests/test_pipeline_gpu.py -k "lora or batch or recompute or kl or varlen or adapter or narrow or dp or reproducible or ppo" > gpurun_out/p/tests.log 2>&1
rc=$?; tail -3 gpurun_out/p/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/p/bench_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/p/bench_$i.log
done
