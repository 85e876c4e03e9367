#!/bin/bash
# Round-6 call AD: wide kernel limited to N <= 16384 — kernel tests, decode steps, serving
set -o pipefail
mkdir -p gpurun_out/ad
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py > gpurun_out/ad/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ad/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 32 64; do
  timeout -k 10 300 python3 -u tools/decode_profile.py --batch $b --prompt 173 --new 64 --iters 2 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a gpurun_out/ad/steps.log || exit 1
done
timeout -k 10 900 python -u bench.py --mode serve --serve-concurrency 1,16,32,64 > gpurun_out/ad/serve.log 2>&1 || exit 1
tail -1 gpurun_out/ad/serve.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); [print(l) for l in d['levels']]"
