#!/bin/bash
# Round-6 call Q: run-to-run reproducibility of the atomic vs slab LoRA TN products
set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 300 python -u tools/r6/atomic_vs_slab_repro.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/q/repro.log
