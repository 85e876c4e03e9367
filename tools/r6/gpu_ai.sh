#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ai
timeout -k 10 300 python -u tools/r6/wide_split_sweep.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ai/sweep.log
