#!/bin/bash
# continuous batching over the active-row bucket: tests, serving bench.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py \
  -k "continuous or teacher or graph" > gpurun_out/r3/test_cont2.log 2>&1 || { tail -40 gpurun_out/r3/test_cont2.log; exit 1; }
tail -1 gpurun_out/r3/test_cont2.log
timeout -k 10 500 python3 -u bench.py --mode serve --serve-engine continuous --serve-concurrency 1,4,16,64 --serve-requests 64 > gpurun_out/r3/bench_serve_continuous3.log 2>&1 || { tail -20 gpurun_out/r3/bench_serve_continuous3.log; exit 1; }
grep "serve c=" gpurun_out/r3/bench_serve_continuous3.log
