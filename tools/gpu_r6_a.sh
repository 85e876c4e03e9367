set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_models_gpu.py tests/test_kernels_gpu.py -k "ppo_loss or batch or bitwise or teacher or varlen or adapter or continuous or row_dot or recompute or kl" > gpurun_out/t1.log 2>&1
rc=$?
tail -5 gpurun_out/t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 > gpurun_out/b1.log 2>&1
