#!/bin/bash
# round 5, GPU call D: persistent gemm_big grid (gemm_persist) vs one workgroup per tile, same box,
# interleaved; PPO bench with old_logp recompute (cost of exact theta_old log-probs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5d
mkdir -p $O
for r in 1 2; do
  for v in - persist; do
    echo "== $v" >> $O/persist.log
    timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_base 10 $v >> $O/persist.log 2>&1 || exit 1
  done
done
cat $O/persist.log
timeout -k 10 300 python -u tools/gemm_big_probe.py --M 9632 --cases nt,nn,lib_nt --sweep gemm_persist=1 --rounds 3 > $O/persist_probe.log 2>&1 || exit 2
grep "M=" $O/persist_probe.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 2 --skip-latency --old-logp recompute > $O/bench_recompute.log 2>&1 || { tail -20 $O/bench_recompute.log; exit 3; }
tail -1 $O/bench_recompute.log
