#!/bin/bash
# round 5, GPU call AB: per-kernel times of the batch-1 loop with / without attention weight prefetch
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ab
mkdir -p $O
export TMPDIR=/tmp
for pf in 1 0; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof$pf -o run -- python3 -u bench.py --steps 0 --latency-queries 8 --tuning attn_prefetch=$pf > $O/pf$pf.log 2>&1 || { tail -20 $O/pf$pf.log; exit 1; }
  find /tmp/prof$pf -name "*kernel_stats.csv" -exec cp {} $O/pf${pf}_kernel_stats.csv \;
done
ls -la $O; tail -3 $O/pf1.log
