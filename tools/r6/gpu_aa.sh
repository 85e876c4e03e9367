#!/bin/bash
# Round-6 call AA: wide kernel + fused decode layer to batch 64 — full GPU tier, serving, headline
set -o pipefail
mkdir -p gpurun_out/aa
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/aa/gputests.log 2>&1
rc=$?; tail -3 gpurun_out/aa/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --mode serve --serve-concurrency 1,16,32,64 > gpurun_out/aa/serve.log 2>&1 || exit 1
tail -1 gpurun_out/aa/serve.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); [print(l) for l in d['levels']]"
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/aa/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*\|"p50_rag_latency_s": [0-9.]*' gpurun_out/aa/bench.log
