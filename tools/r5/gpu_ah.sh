#!/bin/bash
# round 5, GPU call AH: batch-256 o / down split-K factor with the slab-summing norm
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ah
mkdir -p $O
cd tools/r5
for r in 1 2; do
timeout -k 10 300 python -u m256_split_norm_probe.py >> ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
done
grep -E "^(o|down):" ../../$O/probe.log
