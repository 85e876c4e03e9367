#!/bin/bash
# end-of-block check: full GPU suite, smoke, default bench, config-5 pipeline bench.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3/gputests4.log 2>&1 || { tail -40 gpurun_out/r3/gputests4.log; exit 1; }
tail -1 gpurun_out/r3/gputests4.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke4.log 2>&1 || { cat gpurun_out/r3/smoke4.log; exit 1; }
tail -1 gpurun_out/r3/smoke4.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/r3/bench_default4.log 2>&1 || { tail -20 gpurun_out/r3/bench_default4.log; exit 1; }
grep -v "^[EW]2026" gpurun_out/r3/bench_default4.log | tail -1 | cut -c1-300
timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline4.log 2>&1 || { tail -20 gpurun_out/r3/bench_pipeline4.log; exit 1; }
grep -v "^[EW]2026" gpurun_out/r3/bench_pipeline4.log | tail -1 | cut -c1-200
grep -o '"ppo_phase_s_per_step.*' gpurun_out/r3/bench_pipeline4.log
