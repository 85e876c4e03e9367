#!/bin/bash
# Round-6 probe L: batch-256 decode GEMMs at padded / power-of-two operand strides, and the
# operand streams in isolation (activations only / weights only).
set -euo pipefail
mkdir -p gpurun_out/l
for b in both xonly wonly; do
  echo "== $b"
  timeout -k 10 120 tools/r6/bin/gemm_m256_pad_$b 256 2>&1 | tee gpurun_out/l/pad_$b.log
done
