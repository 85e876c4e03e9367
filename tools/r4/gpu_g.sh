#!/bin/bash
# round 4, GPU call G: GEMM stall variants (timing only), rope-epilogue / fused rope-backward tests,
# full GPU tier, headline bench with a torch profile of one extra step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
for v in base nowait nobar_end noprio nolgkm nowait_nobar_end nodma noread mfma_bar; do
  echo "== $v" >> gpurun_out/r4/g_gemm_exp.log
  timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> gpurun_out/r4/g_gemm_exp.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r4/g_gemm_exp.log; exit 1; }
done
echo "== base ring" >> gpurun_out/r4/g_gemm_exp.log
timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_base 10 ring >> gpurun_out/r4/g_gemm_exp.log 2>&1 || { echo "ring run failed"; tail -5 gpurun_out/r4/g_gemm_exp.log; exit 1; }
echo "== base again" >> gpurun_out/r4/g_gemm_exp.log
timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_base 10 >> gpurun_out/r4/g_gemm_exp.log 2>&1 || exit 1
cat gpurun_out/r4/g_gemm_exp.log
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread \
  -k "ring" > gpurun_out/r4/g_ring_tests.log 2>&1 || { echo "ring tests failed"; tail -40 gpurun_out/r4/g_ring_tests.log; exit 1; }
tail -2 gpurun_out/r4/g_ring_tests.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread \
  -k "rope" > gpurun_out/r4/g_rope_tests.log 2>&1 || { echo "rope tests failed"; tail -40 gpurun_out/r4/g_rope_tests.log; exit 1; }
tail -2 gpurun_out/r4/g_rope_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/r4/g_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r4/g_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/g_gpu_tests.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --torch-profile gpurun_out/r4/g_torch_profile.txt > gpurun_out/r4/g_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r4/g_bench.log; exit 1; }
grep '^{' gpurun_out/r4/g_bench.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
