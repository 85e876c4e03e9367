#!/bin/bash
# round 5, GPU call AQ: final-tree PPO kernel profile + config-5 pipeline at round 4's step count
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aq
mkdir -p $O
PROF_TAG=prof_ppo_final bash tools/r5/prof_ppo.sh || exit 1
timeout -k 10 600 python -u bench.py --mode pipeline --steps 2 --warmup 1 --skip-latency > $O/pipeline.log 2>&1 || { tail -20 $O/pipeline.log; exit 2; }
python3 -c "import json; d=json.loads(open('$O/pipeline.log').read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],1), d['ppo_phase_s_per_step'], 'sft', round(d['sft']['value'],1))"
