#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/gputests_r35.log 2>&1 || { tail -30 gpurun_out/r3/gputests_r35.log; exit 1; }
tail -2 gpurun_out/r3/gputests_r35.log
timeout -k 10 400 python -u bench.py --skip-latency > gpurun_out/r3/bench_r35.log 2>&1 || { tail -30 gpurun_out/r3/bench_r35.log; exit 1; }
tail -1 gpurun_out/r3/bench_r35.log
