# round 6 call D: direct LoRA grads (tests + bench A/B), divergence trace without adapters
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_batch_invariance_gpu.py tests/test_models_gpu.py tests/test_pipeline_gpu.py -k "lora or ppo or sft or batch or recompute or kl or varlen or adapter" > gpurun_out/t4.log 2>&1
rc=$?; tail -4 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/b_direct.log 2>&1 || exit 1
grep -o '"phase_s_per_step": {[^}]*}' gpurun_out/b_direct.log; grep -o '"value": [0-9.]*' gpurun_out/b_direct.log
timeout -k 10 300 python -u tools/r6/divergence_trace.py --batch 1 --steps 24 --lora 0 > gpurun_out/div_b1_nolora.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/div_b1_nolora.log
