#!/bin/bash
# round 5, GPU call X: batch-256 decode gate / up + SwiGLU, no-split vs split-K + SwiGLU reduce
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x
mkdir -p $O
timeout -k 10 300 python -u tools/r5/gateup_m256_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
timeout -k 10 300 python -u tools/r5/gateup_m256_probe.py >> $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep "F=" $O/probe.log
