#!/bin/bash
# fp8 K/V decode attention A/B on the 13B batch-64 decode: single-wave 3-deep (default), 8-wave kernel, no-NT loads.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r3/trace14
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  rm -rf /tmp/t14
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/t14 -o run -- python3 $R/tools/decode_profile.py --model llama2-13b --fp8 --fp8-kv --batch 64 --prompt 320 --new 64 > $O/$tag.log 2>&1 || { tail $O/$tag.log; exit 1; }
  f=$(find /tmp/t14 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_gaps.py $f --top 4 > $O/${tag}_gaps.txt
  echo "== $tag"; grep attn_decode $O/${tag}_gaps.txt | head -2; grep "iter 2" $O/$tag.log
}
run default
RT_DECODE_FP8_MW=1 run mw8
RT_ATTN_KV_NT=0 run no_nt
rm -rf /tmp/t14
