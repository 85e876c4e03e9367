#!/bin/bash
# round 5, GPU call AI: batch-256 split-K factors (qkv, 13B fp8 o / down)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ai
mkdir -p $O
cd tools/r5
for r in 1 2; do
timeout -k 10 300 python -u m256_split_probe2.py >> ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
done
grep -E "gemm:|fp8:" ../../$O/probe.log
