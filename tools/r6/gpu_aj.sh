#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/aj
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "m64" > gpurun_out/aj/tests.log 2>&1
rc=$?; tail -2 gpurun_out/aj/tests.log; exit $rc
