#!/bin/bash
# round 5, GPU call AO: head-packed dQ backward — tests, timing, step A/B; then the final PPO profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_props_gpu.py \
  -k "flash or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd tools/r5 && timeout -k 10 300 python -u attn_dq_hp_probe.py > ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
cd ../.. && grep us $O/probe.log
for r in 1 2; do
  for m in 1024 0; do
    echo "== attn_dq_hp_maxs=$m" >> $O/bench.log
    timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --skip-latency --tuning attn_dq_hp_maxs=$m >> $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  done
done
grep -E "^==|^\{" $O/bench.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip(), end=' ')
    else:
        d = json.loads(l); print(round(d['value'], 1), round(d['ms_per_step'], 1), {k: round(v, 3) for k, v in d['phase_s_per_step'].items()})"
