#!/bin/bash
# round 5, GPU call AG: speculative first K / V tiles in the small-batch decode attention — tests, latency, kernel time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ag
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "decode_step or decode_attention or fp8kv" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 0 --latency-queries 24 >> $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 1; }
done
grep -E "p50=" $O/lat.log | sed 's/ stages=.*//'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profg -o run -- python3 -u bench.py --steps 0 --latency-queries 8 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find /tmp/profg -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
grep attn_decode $O/kernel_stats.csv | cut -c1-200
