#!/bin/bash
# Usage (GPU box, repo root): tools/decode_prof.sh <batch> [new]  -> gpurun_out/prof_decode_b<batch>/
set -o pipefail
R=$PWD
B=$1; N=${2:-64}
out=$R/gpurun_out/prof_decode_b$B
rm -rf /tmp/pd && mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/pd -o run -- python3 $R/tools/decode_profile.py --batch $B --new $N > $out/log.txt 2>&1
rc=$?
find /tmp/pd -name "*kernel_stats.csv" -exec cp {} $out/ \;
rm -rf /tmp/pd
exit $rc
