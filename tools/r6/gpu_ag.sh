#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ag
timeout -k 10 300 python -u tools/r6/norm_bw_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ag/norm.log
