#!/bin/bash
# Round-6 call X: wide bf16 kernel for 16 < M <= 64 — kernel tests, shape probe
set -o pipefail
mkdir -p gpurun_out/x
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "m64 or gemm_decode" > gpurun_out/x/tests.log 2>&1
rc=$?; tail -3 gpurun_out/x/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r6/m64_wide_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/x/probe.log
