#!/bin/bash
# round 4, GPU call H: 2-phase granule ring (bitwise tests, timing vs two-buffer), attention block
# order probe, sampler / rope tests, full GPU tier, headline bench (+ torch profile) and ring A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 180 \
  --timeout-method thread -k "ring or rope or sampler or writes_every_row" > gpurun_out/r4/h_tests.log 2>&1 || { echo "focused tests failed"; tail -40 gpurun_out/r4/h_tests.log; exit 1; }
tail -2 gpurun_out/r4/h_tests.log
L=gpurun_out/r4/h_gemm_exp.log
for m in "" ring "" ring; do
  echo "== base ${m:-two-buffer}" >> $L
  timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_base 10 $m >> $L 2>&1 || { echo "gemm_exp failed"; tail -5 $L; exit 1; }
done
cat $L
for bs in "32 301" "64 150" "8 1204"; do
  set -- $bs
  timeout -k 10 120 python -u tools/attn_train_probe.py --B $1 --S $2 >> gpurun_out/r4/h_attn_probe.log 2>&1 || { echo "attn probe failed"; tail -5 gpurun_out/r4/h_attn_probe.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r4/h_attn_probe.log
timeout -k 10 300 python -u tools/gemm_big_probe.py --rounds 3 --sweep gemm_ring=0,1 > gpurun_out/r4/h_probe_ring.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r4/h_probe_ring.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/h_probe_ring.log | tail -30
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/r4/h_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r4/h_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r4/h_gpu_tests.log
for t in "" "gemm_ring=1"; do
  tag=${t:-default}
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 ${t:+--tuning $t} \
    $( [ -z "$t" ] && echo --torch-profile gpurun_out/r4/h_torch_profile.txt ) > gpurun_out/r4/h_bench_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/r4/h_bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/r4/h_bench_$tag.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench $tag', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
done
