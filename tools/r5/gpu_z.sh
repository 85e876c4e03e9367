#!/bin/bash
# round 5, GPU call Z: batch-1 GEMVs cold vs Infinity-Cache-warm weights
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5z
mkdir -p $O
cd tools/r5
timeout -k 10 300 python -u gemv_warm_probe.py > ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
timeout -k 10 300 python -u gemv_warm_probe.py >> ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
cat ../../$O/probe.log
