#!/bin/bash
# continuous batching: GPU tests (generation / models), then serving bench continuous vs dynamic.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py tests/test_pipeline_gpu.py \
  tests/test_kernels_gpu.py -k "continuous or generation or decode or teacher or graph" > gpurun_out/r3/test_cont.log 2>&1 || { tail -40 gpurun_out/r3/test_cont.log; exit 1; }
tail -1 gpurun_out/r3/test_cont.log
for e in continuous dynamic; do
  timeout -k 10 500 python3 -u bench.py --mode serve --serve-engine $e --serve-concurrency 1,16,64 --serve-requests 64 > gpurun_out/r3/bench_serve_$e.log 2>&1 || { tail -20 gpurun_out/r3/bench_serve_$e.log; exit 1; }
  echo "== $e"; grep "serve c=" gpurun_out/r3/bench_serve_$e.log
done
