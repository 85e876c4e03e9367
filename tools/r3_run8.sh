#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 120 python3 -u tools/w4_debug.py > gpurun_out/r3/w4_debug.log 2>&1; rc=$?
cat gpurun_out/r3/w4_debug.log
exit $rc
