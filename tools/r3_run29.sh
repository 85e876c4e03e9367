#!/bin/bash
# host-side cProfile of PPO steps: where the 0.9 s "ref_logprobs+reward" wall time goes when its
# kernels take 0.2 s
set -o pipefail
mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m cProfile -o gpurun_out/r3/bench_cprofile.prof bench.py --steps 2 --warmup 1 --skip-latency > gpurun_out/r3/bench_cprofile.log 2>&1 || { tail -20 gpurun_out/r3/bench_cprofile.log; exit 1; }
python3 - <<'PY' > gpurun_out/r3/bench_cprofile_top.txt
import pstats
s = pstats.Stats("gpurun_out/r3/bench_cprofile.prof")
s.sort_stats("cumulative").print_stats(70)
s.print_callees("prepare")
s.print_callees("_collect_rewards")
s.print_callees("score")
PY
tail -1 gpurun_out/r3/bench_cprofile.log
