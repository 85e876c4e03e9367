#!/bin/bash
# Round-6 probe M: load-only K/V stream of the batch-256 decode attention pattern (tools/r6/kv_stream_probe.hip)
set -euo pipefail
mkdir -p gpurun_out/m
timeout -k 10 120 tools/r6/bin/kv_stream_probe 2>&1 | tee gpurun_out/m/kv_stream_probe.log
