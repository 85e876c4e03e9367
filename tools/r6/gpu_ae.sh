#!/bin/bash
# Round-6 call AE: 4-wave SwiGLU wide form at 16 < M <= 64 — tests, probe
set -o pipefail
mkdir -p gpurun_out/ae
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "m64" > gpurun_out/ae/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ae/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/r6/m64_wide_probe.py 24,32,64 2>&1 | grep -v amdgpu.ids | grep "gate_up\|total" | tee gpurun_out/ae/probe.log
