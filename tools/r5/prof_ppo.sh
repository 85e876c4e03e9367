#!/bin/bash
# Headline PPO step under rocprofv3 (kernel + marker trace) with phase-synchronised roctx ranges
# (RAGTL_PHASE_SYNC=1): per-phase kernel tables whose totals match the bench's phase timers.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5/${PROF_TAG:-prof_ppo}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export RAGTL_PHASE_SYNC=1
timeout -k 10 700 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d /tmp/pp -o run -- \
  python3 $R/bench.py --steps ${STEPS:-2} --warmup 1 --skip-latency > $OUT/log.txt 2>&1 || exit $?
python3 $R/tools/phase_breakdown.py /tmp/pp --top 30 --out $OUT/phases.json > $OUT/phases.txt 2>&1
find /tmp/pp -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
rm -rf /tmp/pp
tail -2 $OUT/log.txt
head -5 $OUT/phases.txt
