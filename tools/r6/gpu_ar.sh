#!/bin/bash
# Round-6 call AR: rocprofv3 kernel + marker trace of the headline PPO step on the current tree
# (phase-synchronised roctx ranges), per-kernel stats and per-phase attribution.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ar
RAGTL_PHASE_SYNC=1 timeout -k 10 900 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d /tmp/profppo -o run \
  -- python3 -u $R/bench.py --steps 3 --warmup 1 --skip-latency > $R/gpurun_out/ar/bench.log 2>&1
rc=$?; tail -3 $R/gpurun_out/ar/bench.log; [ $rc -eq 0 ] || exit $rc
cp $(find /tmp/profppo -name '*kernel_stats.csv' | head -1) $R/gpurun_out/ar/ppo_kernel_stats.csv
python3 $R/tools/phase_breakdown.py /tmp/profppo --top 30 > $R/gpurun_out/ar/ppo_phases.txt
grep -o '"value": [0-9.]*\|"phase_s_per_step": {[^}]*}' $R/gpurun_out/ar/bench.log
