#!/bin/bash
# Round-6 call AU: continuous-batching RAG serving at 128 / 256 concurrent clients (decode rows past
# the fused-layer / wide-kernel range: the split-K token-parallel GEMMs), final tree.
set -o pipefail
mkdir -p gpurun_out/au
timeout -k 10 900 python -u bench.py --mode serve --serve-concurrency 64,128,256 --serve-requests 512 > gpurun_out/au/serve.log 2>&1
rc=$?; grep '\[bench\] serve' gpurun_out/au/serve.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/au/serve.log; exit $rc; }
