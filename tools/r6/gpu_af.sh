#!/bin/bash
# Round-6 call AF: secondary modes on the final tree (config 3 SFT, config 5 pipeline, full-FT PPO)
set -o pipefail
mkdir -p gpurun_out/af
timeout -k 10 600 python -u bench.py --mode sft --steps 3 --warmup 1 > gpurun_out/af/sft.log 2>&1 || exit 1
tail -1 gpurun_out/af/sft.log | cut -c1-200
timeout -k 10 900 python -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/af/pipe.log 2>&1 || exit 1
grep -o '"metric": "[^"]*", "value": [0-9.]*' gpurun_out/af/pipe.log
timeout -k 10 900 python -u bench.py --full-ft --steps 2 --warmup 1 --skip-latency > gpurun_out/af/fullft.log 2>&1 || exit 1
tail -1 gpurun_out/af/fullft.log | cut -c1-200
