#!/bin/bash
# round 5, GPU call AC: batch-1 GEMV knobs (waves, depth) from cold weights
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ac
mkdir -p $O
cd tools/r5
for r in 1 2; do
timeout -k 10 300 python -u gemv_knob_probe.py >> ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
done
grep MB ../../$O/probe.log
