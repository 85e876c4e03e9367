#!/bin/bash
# Batch-256 bf16 decode (Mistral-7B) and batch-64 fp8 decode (Llama-2-13B): kernel traces + gaps.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r3/trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/td256 -o run -- python3 $R/tools/decode_profile.py --batch 256 --prompt 173 --new 64 > $O/b256_log.txt 2>&1 || { tail $O/b256_log.txt; exit 1; }
f=$(find /tmp/td256 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f --top 20 > $O/b256_gaps.txt
cat $O/b256_gaps.txt
grep iter $O/b256_log.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/td64 -o run -- python3 $R/tools/decode_profile.py --model llama2-13b --fp8 --batch 64 --prompt 320 --new 64 > $O/b64_13b_log.txt 2>&1 || { tail $O/b64_13b_log.txt; exit 1; }
f=$(find /tmp/td64 -name "*kernel_trace.csv" | head -1)
python3 $R/tools/trace_gaps.py $f --top 20 > $O/b64_13b_gaps.txt
cat $O/b64_13b_gaps.txt
grep iter $O/b64_13b_log.txt
rm -rf /tmp/td256 /tmp/td64
