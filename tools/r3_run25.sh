#!/bin/bash
# DP rehearsal on one GPU: 2 ranks over gloo (RCCL needs one GPU per rank), headline bench path.
set -o pipefail
mkdir -p gpurun_out/r3
export RAGTL_DIST_BACKEND=gloo
timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 1 --warmup 1 --rollout-batch 64 --skip-latency > gpurun_out/r3/bench_dp2_gloo.log 2>&1 || { tail -30 gpurun_out/r3/bench_dp2_gloo.log; exit 1; }
grep -v "^[EW]2026\|amdgpu.ids\|socket.cpp" gpurun_out/r3/bench_dp2_gloo.log | tail -3 | cut -c1-700
