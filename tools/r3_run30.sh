#!/bin/bash
# kernel + copy + marker trace of a 2-step bench: GPU idle gaps per phase
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/r3/idle
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace -f csv -d /tmp/ti -o run -- python3 $R/bench.py --steps 1 --warmup 1 --skip-latency > $R/gpurun_out/r3/idle/log.txt 2>&1 || exit $?
python3 $R/tools/timeline_idle.py /tmp/ti --last-frac 0.45 > $R/gpurun_out/r3/idle/gaps.txt 2>&1
python3 $R/tools/phase_breakdown.py /tmp/ti --top 12 > $R/gpurun_out/r3/idle/phases.txt 2>&1
head -30 $R/gpurun_out/r3/idle/gaps.txt
rm -rf /tmp/ti
