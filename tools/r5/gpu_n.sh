#!/bin/bash
# round 5, GPU call N: full GPU tier + smoke + batch-1 latency with the faster top-k sampler
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 0 --latency-queries 16 > $O/lat.log 2>&1 || { tail -20 $O/lat.log; exit 3; }
tail -1 $O/lat.log | cut -c1-300
