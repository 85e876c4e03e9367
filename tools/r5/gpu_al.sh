#!/bin/bash
# round 5, GPU call AL: LoRA narrow-product split sweep at the update shape
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5al
mkdir -p $O
cd tools/r5
timeout -k 10 400 python -u lora_narrow_sweep.py > ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
grep -E "^(U|dU|dA|dB) " ../../$O/probe.log
