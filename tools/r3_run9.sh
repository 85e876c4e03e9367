#!/bin/bash
# Round-3 re-entry: full GPU suite, smoke, default bench, 4-wave GEMM numerics.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3/gputests.log 2>&1 || { tail -40 gpurun_out/r3/gputests.log; exit 1; }
tail -3 gpurun_out/r3/gputests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke.log 2>&1 || { cat gpurun_out/r3/smoke.log; exit 1; }
tail -1 gpurun_out/r3/smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3/bench.log 2>&1 || { tail -20 gpurun_out/r3/bench.log; exit 1; }
tail -2 gpurun_out/r3/bench.log
timeout -k 10 120 python3 -u tools/w4_debug.py > gpurun_out/r3/w4_debug.log 2>&1; rc=$?
grep "bn=" gpurun_out/r3/w4_debug.log
exit 0
