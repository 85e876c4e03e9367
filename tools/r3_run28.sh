#!/bin/bash
# re-entry check of the restored tree: full GPU suite, smoke, default headline bench.
set -o pipefail
mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/gputests_reentry3.log 2>&1 || { tail -30 gpurun_out/r3/gputests_reentry3.log; exit 1; }
tail -3 gpurun_out/r3/gputests_reentry3.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3/smoke_reentry3.log 2>&1 || { tail -20 gpurun_out/r3/smoke_reentry3.log; exit 1; }
tail -1 gpurun_out/r3/smoke_reentry3.log
timeout -k 10 400 python -u bench.py > gpurun_out/r3/bench_default_reentry3.log 2>&1 || { tail -30 gpurun_out/r3/bench_default_reentry3.log; exit 1; }
tail -1 gpurun_out/r3/bench_default_reentry3.log
