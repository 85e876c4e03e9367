#!/bin/bash
# round 5, GPU call Y: batch-1 GEMV time vs workgroups per CU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 300 python -u tools/r5/gemv_balance_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
timeout -k 10 300 python -u tools/r5/gemv_balance_probe.py >> $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
