#!/bin/bash
# Round-6 call W: decode step time vs batch (serving sizes 16 / 32 / 48 / 64 and the rollout's 256), kernel stats at 64
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/w
for b in 16 32 64 128 256; do
  timeout -k 10 300 python3 -u $R/tools/decode_profile.py --batch $b --prompt 173 --new 64 --iters 2 2>&1 | grep -v amdgpu.ids | tail -2 | tee -a $R/gpurun_out/w/steps.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/profw -o run -- python3 -u $R/tools/decode_profile.py --batch 64 --prompt 173 --new 64 --iters 1 > $R/gpurun_out/w/prof.log 2>&1 || exit 1
cp $(find /tmp/profw -name '*kernel_stats.csv' | head -1) $R/gpurun_out/w/b64_kernel_stats.csv
