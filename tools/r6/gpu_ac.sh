#!/bin/bash
# Round-6 call AC: M <= 64 probe incl. the LM head
set -o pipefail
mkdir -p gpurun_out/ac
timeout -k 10 300 python -u tools/r6/m64_wide_probe.py 32,64 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ac/probe.log
