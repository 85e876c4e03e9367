#!/bin/bash
# Round-6 call S: bitwise reproducibility / resume tests
set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batch_invariance_gpu.py > gpurun_out/s/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/s/tests.log | tail -30; exit $rc
