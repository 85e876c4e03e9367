#!/bin/bash
# Round-6 call AN: re-tuned LoRA narrow-product splits — tests, headline bench x2
set -o pipefail
mkdir -p gpurun_out/an
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_kernels_gpu.py tests/test_zz_dist_gpu.py -k "lora or reproducible or resume or narrow or dp" > gpurun_out/an/tests.log 2>&1
rc=$?; tail -2 gpurun_out/an/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/an/bench_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/an/bench_$i.log
done
