#!/bin/bash
# full GPU suite + smoke on the current tree, then the serving bench (dynamic batching).
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3/gputests2.log 2>&1 || { tail -40 gpurun_out/r3/gputests2.log; exit 1; }
tail -1 gpurun_out/r3/gputests2.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke2.log 2>&1 || { cat gpurun_out/r3/smoke2.log; exit 1; }
tail -1 gpurun_out/r3/smoke2.log
timeout -k 10 500 python3 -u bench.py --mode serve --serve-concurrency 1,4,16 --serve-requests 48 > gpurun_out/r3/bench_serve.log 2>&1 || { tail -20 gpurun_out/r3/bench_serve.log; exit 1; }
grep "serve c=" gpurun_out/r3/bench_serve.log
