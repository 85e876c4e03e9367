#!/bin/bash
# Round-6 call R: fixed-order norm weight / embedding gradients — full GPU tier, then the
# full-fine-tuning bench (the path those gradients are on) and the headline bench
set -o pipefail
mkdir -p gpurun_out/r
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/r/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --full-ft --steps 2 --warmup 1 --skip-latency > gpurun_out/r/bench_fullft.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/r/bench_fullft.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency > gpurun_out/r/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/r/bench.log
