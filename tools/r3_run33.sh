#!/bin/bash
# LoRA narrow products: kernel-only durations (rocprof stats) of the probe shapes
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/r3/narrow
timeout -k 10 200 python3 -u tools/lora_narrow_probe.py > $R/gpurun_out/r3/narrow/probe.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/nw -o run -- python3 $R/tools/lora_narrow_probe.py --rounds 1 > $R/gpurun_out/r3/narrow/prof_log.txt 2>&1 || exit $?
find /tmp/nw -name "*kernel_trace.csv" -exec cp {} $R/gpurun_out/r3/narrow/trace.csv \;
find /tmp/nw -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r3/narrow/kernel_stats.csv \;
rm -rf /tmp/nw
cat $R/gpurun_out/r3/narrow/probe.log
