#!/bin/bash
# round 5, GPU call AR: the other bench modes on the final round-5 kernels — SFT (config 3),
# full-parameter PPO, serving (continuous batching), PPO with 1-3 retrieved docs per query
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ar
mkdir -p $O
run() {  # tag, timeout, args...
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > $O/$tag.log 2>&1 || { echo "bench $tag failed"; tail -20 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log | tail -1 | cut -c1-300
}
run sft 400 --mode sft --steps 5 --warmup 2 --skip-latency
run fullft 600 --full-ft --steps 3 --warmup 1 --skip-latency
run serve 500 --mode serve --serve-concurrency 1,16,64 --serve-requests 64
run varydocs 500 --vary-docs --steps 4 --warmup 2 --skip-latency
