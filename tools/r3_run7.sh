#!/bin/bash
# 4-wave NT GEMM tiles: numerics, then A/B timing vs the 8-wave kernel and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 120 python3 -u tools/w4_debug.py > gpurun_out/r3/w4_debug.log 2>&1 || { cat gpurun_out/r3/w4_debug.log; exit 1; }
grep "bn=" gpurun_out/r3/w4_debug.log
timeout -k 10 240 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_big_gpu.py -k "w4" \
  > gpurun_out/r3/test_w4.log 2>&1 || { tail -30 gpurun_out/r3/test_w4.log; exit 1; }
tail -3 gpurun_out/r3/test_w4.log
timeout -k 10 400 python3 tools/gemm_big_probe.py --M 9632 --shapes qkv,o,gate_up,down \
  --cases nt,w4_192,w4_256,lib_nt,nt_swiglu,w4_192_swiglu,w4_256_swiglu --rounds 5 > gpurun_out/r3/w4_probe.log 2>&1
cat gpurun_out/r3/w4_probe.log
timeout -k 10 200 python3 tools/gemm_big_probe.py --M 256 --shapes qkv,o,gate_up,down \
  --cases nt128,w4_192,w4_256,lib_nt,nt128_swiglu,w4_192_swiglu --rounds 3 > gpurun_out/r3/w4_probe_m256.log 2>&1
cat gpurun_out/r3/w4_probe_m256.log
