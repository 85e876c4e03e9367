#!/bin/bash
# final-tree evidence: rocprofv3 kernel stats + per-phase breakdown of a headline PPO step, then the
# config-5 (Llama-2-13B fp8) pipeline bench
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/r3/final_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d /tmp/fp -o run -- python3 $R/bench.py --steps 1 --warmup 1 --skip-latency > $R/gpurun_out/r3/final_prof/log.txt 2>&1 || exit $?
python3 $R/tools/phase_breakdown.py /tmp/fp --top 25 > $R/gpurun_out/r3/final_prof/phases.txt 2>&1
find /tmp/fp -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r3/final_prof/kernel_stats.csv \;
rm -rf /tmp/fp
cd $R
timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline13b_final.log 2>&1 || { tail -20 gpurun_out/r3/bench_pipeline13b_final.log; exit 1; }
tail -1 gpurun_out/r3/bench_pipeline13b_final.log
