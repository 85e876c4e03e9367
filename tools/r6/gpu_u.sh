#!/bin/bash
# Round-6 call U: serving (continuous batching) and variable-docs PPO on the final tree
set -o pipefail
mkdir -p gpurun_out/u
timeout -k 10 900 python -u bench.py --mode serve --steps 3 --warmup 1 > gpurun_out/u/serve.log 2>&1 || exit 1
tail -1 gpurun_out/u/serve.log | cut -c1-400
timeout -k 10 900 python -u bench.py --vary-docs --steps 3 --warmup 1 --skip-latency > gpurun_out/u/varydocs.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/u/varydocs.log
