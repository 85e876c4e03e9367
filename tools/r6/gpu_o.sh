#!/bin/bash
# Round-6 call O: full GPU tier + smoke on the final tree, then a 20-step headline bench.
set -o pipefail
mkdir -p gpurun_out/o
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/o/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/o/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/o/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/o/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/o/bench20.log 2>&1
rc=$?; grep -o '"value": [0-9.]*\|"p50_rag_latency_s": [0-9.]*\|"phase_s_per_step": {[^}]*}' gpurun_out/o/bench20.log; exit $rc
