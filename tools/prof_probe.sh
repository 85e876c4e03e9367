#!/bin/bash
# Kernel-trace stats of tools/gemm_big_probe.py (args passed through) -> gpurun_out/prof_probe/
set -o pipefail
R=$PWD
out=$R/gpurun_out/prof_probe
rm -rf /tmp/pp_probe && mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d /tmp/pp_probe -o run -- python3 $R/tools/gemm_big_probe.py "$@" > $out/log.txt 2>&1
rc=$?
find /tmp/pp_probe -name "*kernel_stats.csv" -exec cp {} $out/ \;
rm -rf /tmp/pp_probe
exit $rc
