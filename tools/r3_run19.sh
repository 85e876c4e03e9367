#!/bin/bash
# row-bucketed decode graphs: generation/model GPU tests, serving bench, default headline bench.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3/gputests3.log 2>&1 || { tail -40 gpurun_out/r3/gputests3.log; exit 1; }
tail -1 gpurun_out/r3/gputests3.log
timeout -k 10 500 python3 -u bench.py --mode serve --serve-concurrency 1,4,16,64 --serve-requests 64 > gpurun_out/r3/bench_serve2.log 2>&1 || { tail -20 gpurun_out/r3/bench_serve2.log; exit 1; }
grep "serve c=" gpurun_out/r3/bench_serve2.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/r3/bench_default2.log 2>&1 || { tail -20 gpurun_out/r3/bench_default2.log; exit 1; }
grep -v "^[EW]2026" gpurun_out/r3/bench_default2.log | tail -1 | cut -c1-400
