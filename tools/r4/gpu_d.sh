#!/bin/bash
# round 4, GPU call D: (1) bench.py --gpus 2 self-launch rehearsal over gloo on one GPU,
# (2) reference-scoring chunk A/B (64 vs 256 sequences per forward), (3) config-5 batch sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "norm" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4/d_norm_tests.log 2>&1 || { echo "norm tests failed"; tail -30 gpurun_out/r4/d_norm_tests.log; exit 1; }
tail -1 gpurun_out/r4/d_norm_tests.log
timeout -k 10 120 python -u tools/r4/norm_slab_probe.py > gpurun_out/r4/d_norm_probe.log 2>&1 && grep -v amdgpu.ids gpurun_out/r4/d_norm_probe.log
RAGTL_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 1 --warmup 1 --skip-latency \
  > gpurun_out/r4/d_bench_gpus2_gloo.log 2>&1 || { echo "gloo 2-rank bench failed"; tail -30 gpurun_out/r4/d_bench_gpus2_gloo.log; exit 1; }
grep '^{' gpurun_out/r4/d_bench_gpus2_gloo.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('gloo2', r['n_gpus'], r['world'], r['value'], r['allreduce_probe'])"
for rm in 64 256; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --skip-latency --ref-minibatch $rm \
    > gpurun_out/r4/d_bench_ref$rm.log 2>&1 || { echo "bench ref$rm failed"; tail -20 gpurun_out/r4/d_bench_ref$rm.log; exit 1; }
  grep '^{' gpurun_out/r4/d_bench_ref$rm.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('ref_mb=$rm', round(r['value']), round(r['ms_per_step']), r['phase_s_per_step'])"
done
bash tools/r4/gpu_c.sh
