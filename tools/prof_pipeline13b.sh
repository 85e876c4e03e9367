#!/bin/bash
# rocprofv3 kernel statistics + per-phase breakdown (roctx PhaseTimer ranges) of the config-5
# pipeline bench (Llama-2-13B, fp8 inference GEMMs): SFT step + PPO step (rollout, reference
# scoring, update). Kernel trace + marker trace + stats only (no counters).
# Usage (GPU box, repo root): bash tools/prof_pipeline13b.sh [extra bench args]
set -o pipefail
R=$PWD
out=$R/gpurun_out/prof13b
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/p13b
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d /tmp/p13b -o run -- python3 $R/bench.py \
  --mode pipeline --steps 1 --warmup 1 "$@" > $out/bench.log 2>&1 || exit $?
python3 $R/tools/phase_breakdown.py /tmp/p13b --top 25 > $out/phases.txt 2>&1
find /tmp/p13b -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
rm -rf /tmp/p13b
ls -la $out
