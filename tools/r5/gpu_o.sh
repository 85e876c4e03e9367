#!/bin/bash
# round 5, GPU call O: headline A/B of the reference-scoring minibatch (64 default, 128, 256)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5o
mkdir -p $O
for rm in 64 128 256 64; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --skip-latency --ref-minibatch $rm > $O/bench_ref$rm.log 2>&1 || { tail -20 $O/bench_ref$rm.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_ref$rm.log').read().strip().splitlines()[-1]); print('ref_mb $rm', round(d['value'],1), {k: round(v,3) for k,v in d['phase_s_per_step'].items() if k.startswith('time/')})"
done
