#!/bin/bash
# round 4, GPU call N: 8-wave attention forward (bitwise test, probe A/B, bench A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread \
  -k "8wave or flash or attention" > gpurun_out/r4/n_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4/n_tests.log; exit 1; }
tail -2 gpurun_out/r4/n_tests.log
for t in "" attn_fwd_w8=1 "" attn_fwd_w8=1; do
  for bs in "32 301" "64 150" "8 1204"; do
    set -- $bs
    timeout -k 10 120 python -u tools/attn_train_probe.py --B $1 --S $2 ${t:+--tuning $t} >> gpurun_out/r4/n_attn_probe.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r4/n_attn_probe.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r4/n_attn_probe.log
for t in "" "attn_fwd_w8=1"; do
  tag=${t:-default}
  timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 ${t:+--tuning $t} > gpurun_out/r4/n_bench_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/r4/n_bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/r4/n_bench_$tag.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench $tag', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
done
