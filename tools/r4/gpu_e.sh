#!/bin/bash
# round 4, GPU call E: full GPU tier (fused MLP node, slab norm), MLP fwd+bwd probe, headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/r4/e_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r4/e_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/e_gpu_tests.log
timeout -k 10 300 python -u tools/r4/mlp_bwd_probe.py > gpurun_out/r4/e_mlp_probe.log 2>&1 && grep -v amdgpu.ids gpurun_out/r4/e_mlp_probe.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/r4/e_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4/e_bench.log; exit 1; }
grep '^{' gpurun_out/r4/e_bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
