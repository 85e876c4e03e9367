#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/am
timeout -k 10 300 python -u tools/r6/lora_narrow_sweep.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/am/sweep.log
