#!/bin/bash
# round 5, GPU call AS: reference scoring minibatch 128 vs 256 sequences
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5as
mkdir -p $O
for r in 1 2; do
  for m in 256 128; do
    echo "== ref-minibatch $m" >> $O/bench.log
    timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --skip-latency --ref-minibatch $m >> $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  done
done
grep -E "^==|^\{" $O/bench.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip(), end=' ')
    else:
        d = json.loads(l); print(round(d['value'], 1), round(d['ms_per_step'], 1), {k: round(v, 3) for k, v in d['phase_s_per_step'].items()})"
