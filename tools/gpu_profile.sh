#!/bin/bash
# Usage (on the GPU box, from the repo root): tools/gpu_profile.sh <name> <bench args...>
# Kernel trace + stats of one bench invocation; keeps only the *_stats.csv summaries under
# gpurun_out/prof_<name>/ (the raw trace is deleted to stay under the copy-back limit).
set -o pipefail
R=$PWD
name=$1; shift
out=$R/gpurun_out/prof_$name
rm -rf /tmp/prof_$name && mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $out/log.txt 2>&1
rc=$?
find /tmp/prof_$name -name "*stats.csv" -exec cp {} $out/ \;
rm -rf /tmp/prof_$name
echo "profile $name rc=$rc"
exit $rc
