#!/bin/bash
# round 5, GPU call U: config-5 pipeline with deferred (W8A8 split-K) vs reduced decode GEMMs,
# generated tokens per step (EOS) and step time
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5u
mkdir -p $O
for d in off on off on; do
  timeout -k 10 600 python -u bench.py --mode pipeline --steps 3 --warmup 1 --skip-latency --defer-splitk $d > $O/bench_$d.log 2>&1 || { tail -20 $O/bench_$d.log; exit 2; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$d.log') if l.startswith('{')][-1]); print('defer $d', round(d['value'],1), round(d['ms_per_step'],1), 'tok/step', round(d['value']*d['ms_per_step']/1e3), d['ppo_phase_s_per_step'])"
done
