# round 6 call J: fixed-order slab split of the forward LoRA U product — tests + bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_zz_dist_gpu.py -k "lora or batch or recompute or kl or varlen or adapter or narrow or dp" > gpurun_out/t5.log 2>&1
rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/b_uslab_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/b_uslab_$i.log
done
