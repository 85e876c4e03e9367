#!/bin/bash
# Round-6 probe K: wave-specialised batch-256 decode GEMM variants (tools/gemm_exp/gemm_m256ws.hip)
# against gemm_big's 256x128 split-K / SwiGLU forms, bitwise check + timing per shape.
set -euo pipefail
mkdir -p gpurun_out/k
for b in x3w4n0 x3w4n1 x2w6n0 x2w6n1; do
  echo "== $b"
  timeout -k 10 90 tools/r6/bin/gemm_m256ws_$b 256 2>&1 | tee gpurun_out/k/m256ws_$b.log
done
