#!/bin/bash
# Round-6 call Z: bf16 fused decode layer (folded norms, residual epilogues) up to batch 64 vs 16
set -o pipefail
mkdir -p gpurun_out/z
for b in 24 32 64; do
  for fm in 16 64; do
    echo "batch $b fused_max $fm" | tee -a gpurun_out/z/steps.log
    timeout -k 10 300 python3 -u tools/decode_profile.py --batch $b --prompt 173 --new 64 --iters 2 --fused-max $fm 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a gpurun_out/z/steps.log || exit 1
  done
done
