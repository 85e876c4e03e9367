# round 6 call B: sampler fast-path / race fix tests, MFMA power probe, reward-encoder A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py tests/test_kernels_gpu.py -k "sampler or ppo_loss or sample or batch or row_dot or recompute or kl" > gpurun_out/t2.log 2>&1
rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/r6/mfma_probe > gpurun_out/mfma_probe.log 2>&1 || exit 1
cat gpurun_out/mfma_probe.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/b_mpnet.log 2>&1 || exit 1
tail -1 gpurun_out/b_mpnet.log | cut -c1-600
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency --reward-encoder same > gpurun_out/b_minilm.log 2>&1 || exit 1
tail -1 gpurun_out/b_minilm.log | cut -c1-600
