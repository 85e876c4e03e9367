#!/bin/bash
# Round-6 call T: SFT bitwise resume
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py -k "sft" > gpurun_out/t/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/t/tests.log | tail -30; exit $rc
