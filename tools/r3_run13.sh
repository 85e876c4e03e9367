#!/bin/bash
# fp8 K/V decode attention (3-deep prefetch): numerics, then 13B batch-64 kernel durations bf16 vs fp8 cache.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r3/trace13
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8kv or kv_store_fp8" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
cd /tmp && export TMPDIR=/tmp
for kv in "" "--fp8-kv"; do
  tag=kv${kv:-bf16}
  rm -rf /tmp/t13
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/t13 -o run -- python3 $R/tools/decode_profile.py --model llama2-13b --fp8 $kv --batch 64 --prompt 320 --new 64 > $O/$tag.log 2>&1 || { tail $O/$tag.log; exit 1; }
  f=$(find /tmp/t13 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_gaps.py $f --top 8 > $O/${tag}_gaps.txt
  head -10 $O/${tag}_gaps.txt
  grep iter $O/$tag.log
done
rm -rf /tmp/t13
