#!/bin/bash
# round 5, GPU call AP: config-5 pipeline (13B fp8) with / without the short-sequence attention tiles
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ap
mkdir -p $O
for m in 1024 0; do
  echo "== attn_fwd_hp_maxs=$m" >> $O/bench.log
  timeout -k 10 600 python -u bench.py --mode pipeline --steps 3 --warmup 1 --skip-latency --tuning attn_fwd_hp_maxs=$m >> $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 2; }
done
grep -E "^==|^\{" $O/bench.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip(), end=' ')
    else:
        d = json.loads(l); print(round(d['value'], 1), d.get('ppo_phase_s_per_step'), 'sft', round(d['sft']['value'], 1))"
