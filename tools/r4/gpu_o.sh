#!/bin/bash
# round 4, GPU call O: the other bench modes on the late round-4 tree (after the RoPE / SwiGLU-backward fusions) — SFT (config 3), the Llama-2-13B
# pipeline (config 5), full-parameter PPO, serving (continuous batching)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
run() {  # tag, timeout, args...
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > gpurun_out/r4/o_$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/r4/o_$tag.log; exit 1; }
  grep '^{' gpurun_out/r4/o_$tag.log | tail -1 | cut -c1-400
}
run sft 400 --mode sft --steps 5 --warmup 2 --skip-latency
run pipeline13b 700 --mode pipeline --steps 2 --warmup 1 --skip-latency
run fullft 600 --full-ft --steps 3 --warmup 1 --skip-latency
run serve 500 --mode serve --serve-concurrency 1,16,64 --serve-requests 64
