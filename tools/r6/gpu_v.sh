#!/bin/bash
# Round-6 call V: serving at 1 / 16 / 64 concurrent clients (the round-5 README levels)
set -o pipefail
mkdir -p gpurun_out/v
timeout -k 10 900 python -u bench.py --mode serve --serve-concurrency 1,16,64 > gpurun_out/v/serve.log 2>&1 || exit 1
tail -1 gpurun_out/v/serve.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); [print(l) for l in d['levels']]"
