#!/bin/bash
# Kernel statistics of PPO-update minibatches (tools/update_probe.py) -> gpurun_out/prof_update/
set -o pipefail
R=$PWD
out=$R/gpurun_out/prof_update
rm -rf /tmp/pu && mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/pu -o run -- python3 $R/tools/update_probe.py "$@" > $out/log.txt 2>&1
rc=$?
find /tmp/pu -name "*kernel_stats.csv" -exec cp {} $out/ \;
rm -rf /tmp/pu
exit $rc
