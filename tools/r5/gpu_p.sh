#!/bin/bash
# round 5, GPU call P: config-5 pipeline (Llama-2-13B fp8) kernel profile, one PPO step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r5p
mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 -u $GRAFT_REPO_ROOT/bench.py --mode pipeline --steps 1 --warmup 1 --skip-latency > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
head -25 $O/prof/p_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
