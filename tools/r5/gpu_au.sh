#!/bin/bash
# round 5, GPU call AU: L2 tile-group height at the reference / prefill row counts (38528, 44288)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5au
mkdir -p $O
timeout -k 10 500 python -u tools/gemm_big_probe.py --M 38528 44288 --cases nt --sweep gemm_group_m=2,8,16 --rounds 3 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log | tail -30
