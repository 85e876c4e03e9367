#!/bin/bash
# Round-6 call AH: kernel table of the batch-64 decode step on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ah
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/profah -o run -- python3 -u $R/tools/decode_profile.py --batch 64 --prompt 173 --new 64 --iters 1 > $R/gpurun_out/ah/prof.log 2>&1 || exit 1
cp $(find /tmp/profah -name '*kernel_stats.csv' | head -1) $R/gpurun_out/ah/b64_kernel_stats.csv
