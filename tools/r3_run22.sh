#!/bin/bash
# VALU MHA fp8 decode attention: numerics (fp8kv tests cover G = 1 at batch 64), 13B decode A/B vs the MFMA form.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r3/trace22
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8kv or kv_store_fp8" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -1 $O/test.log
cd /tmp && export TMPDIR=/tmp
run() {
  tag=$1; shift
  rm -rf /tmp/t22
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/t22 -o run -- python3 $R/tools/decode_profile.py --model llama2-13b --fp8 --fp8-kv --batch 64 --prompt 320 --new 64 > $O/$tag.log 2>&1 || { tail $O/$tag.log; exit 1; }
  f=$(find /tmp/t22 -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_gaps.py $f --top 6 > $O/${tag}_gaps.txt
  echo "== $tag"; grep attn_decode $O/${tag}_gaps.txt | head -2; grep "iter 2" $O/$tag.log
}
RT_DECODE_G1_NW=1 run nw1
run nw2
RT_DECODE_G1_NW=4 run nw4
rm -rf /tmp/t22
