#!/bin/bash
# Round-6 call AT: full GPU tier + smoke on the final tree (heaviest-first causal attention), then
# the driver's bench shape (20 timed steps after 5 warm-up).
set -o pipefail
mkdir -p gpurun_out/at
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/at/gputests.log 2>&1
rc=$?; tail -2 gpurun_out/at/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/at/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/at/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/at/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"p50_rag_latency_s": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/at/bench.log
