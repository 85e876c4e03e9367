#!/bin/bash
# round 5, GPU call S: fp8-KV decode attention fed by split-K slabs vs reduced qkv
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -s -k "deferred_splitk" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -30 $O/tests.log
exit $rc
