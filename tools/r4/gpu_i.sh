#!/bin/bash
# round 4, GPU call I: attention (double-buffered fwd) / rope / sampler tests + probe, same-box A/B
# of the RoPE fusions (bench default / --rope-fusion off / default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 180 \
  --timeout-method thread -k "attention or attn or rope or sampler or flash or decoder" > gpurun_out/r4/i_tests.log 2>&1 || { echo "focused tests failed"; tail -40 gpurun_out/r4/i_tests.log; exit 1; }
tail -2 gpurun_out/r4/i_tests.log
for bs in "32 301" "64 150" "8 1204"; do
  set -- $bs
  timeout -k 10 120 python -u tools/attn_train_probe.py --B $1 --S $2 >> gpurun_out/r4/i_attn_probe.log 2>&1 || { echo "attn probe failed"; tail -5 gpurun_out/r4/i_attn_probe.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r4/i_attn_probe.log
n=0
for t in on off on; do
  n=$((n+1))
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --rope-fusion $t > gpurun_out/r4/i_bench_${n}_$t.log 2>&1 || { echo "bench $t failed"; tail -20 gpurun_out/r4/i_bench_${n}_$t.log; exit 1; }
  grep '^{' gpurun_out/r4/i_bench_${n}_$t.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench rope-fusion $t', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
done
