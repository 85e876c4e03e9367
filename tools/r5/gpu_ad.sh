#!/bin/bash
# round 5, GPU call AD: batch-1 decode attention split over key partitions (last-arriver merge) at short caches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ad
mkdir -p $O
for r in 1 2; do
  for cfg in "decode_mw_smax=1024" "decode_mw_smax=0,decode_mw_kpp=128" "decode_mw_smax=0,decode_mw_kpp=192"; do
    echo "== $cfg" >> $O/lat.log
    timeout -k 10 300 python -u bench.py --steps 0 --latency-queries 16 --tuning $cfg >> $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
  done
done
grep -E "==|p50=" $O/lat.log
