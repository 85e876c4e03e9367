#!/bin/bash
# round 5, GPU call B: GPU tier after the product-kernel cleanup + ZeRO/adamw_apply bindings,
# behaviour-gap probe, GEMM probe (ours vs hipBLASLt), headline bench (merged and unmerged rollouts)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > $O/gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u tools/r5/behaviour_gap_probe.py > $O/behaviour_gap.log 2>&1 || { tail -20 $O/behaviour_gap.log; exit 2; }
grep -v amdgpu.ids $O/behaviour_gap.log
for v in base kji base kji; do
  echo "== $v" >> $O/gemm_order.log
  timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> $O/gemm_order.log 2>&1 || exit 6
done
cat $O/gemm_order.log
timeout -k 10 300 python -u tools/gemm_big_probe.py --M 9632 --cases nt,nn,lib_nt,lib_nn --rounds 3 > $O/gemm_probe.log 2>&1 || exit 3
grep "M=" $O/gemm_probe.log
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 4; }
tail -1 $O/bench_default.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 2 --skip-latency --merged-rollout off > $O/bench_unmerged.log 2>&1 || { tail -20 $O/bench_unmerged.log; exit 5; }
tail -1 $O/bench_unmerged.log
