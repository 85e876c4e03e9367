#!/bin/bash
# round 5, GPU call R: config-5 pipeline bench repeatability + kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5r
mkdir -p $O
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --mode pipeline --steps 3 --warmup 1 --skip-latency > $O/bench$r.log 2>&1 || { tail -20 $O/bench$r.log; exit 2; }
  python3 -c "import json; d=json.loads(open('$O/bench$r.log').read().strip().splitlines()[-1]); print(round(d['value'],1), round(d['ms_per_step'],1), d['ppo_phase_s_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 -u $GRAFT_REPO_ROOT/bench.py --mode pipeline --steps 1 --warmup 1 --skip-latency > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 3; }
echo profiled
