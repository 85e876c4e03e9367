#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py -x -q --timeout 120 --timeout-method thread -k "small_tile" > gpurun_out/r3/test_small_bm.log 2>&1 || { tail -30 gpurun_out/r3/test_small_bm.log; exit 1; }
tail -2 gpurun_out/r3/test_small_bm.log
timeout -k 10 200 python3 -u tools/small_bm_probe.py > gpurun_out/r3/small_bm_probe.log 2>&1 || { tail -20 gpurun_out/r3/small_bm_probe.log; exit 1; }
cat gpurun_out/r3/small_bm_probe.log
