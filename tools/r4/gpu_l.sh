#!/bin/bash
# round 4, GPU call L: 8-wave vs 4-wave (bn = 4) kernels on the update shapes, and the 4-wave kernel
# without its LDS-DMA waits (is it latency-bound?)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
L=gpurun_out/r4/l_gemm_w4.log
for v in "base" "base w4" "w4nowait w4" "base" "base w4" "w4nowait w4"; do
  set -- $v
  echo "== $v" >> $L
  timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$1 10 $2 >> $L 2>&1 || { echo "gemm_exp $v failed"; tail -5 $L; exit 1; }
done
cat $L
