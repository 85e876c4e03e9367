#!/bin/bash
# round 5, GPU call V: 640-thread slab norm (H = 5120): tests + config-5 pipeline (steps 2, as round 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "norm" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --mode pipeline --steps 2 --warmup 1 --skip-latency > $O/bench$r.log 2>&1 || { tail -20 $O/bench$r.log; exit 2; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench$r.log') if l.startswith('{')][-1]); print(round(d['value'],1), round(d['ms_per_step'],1), 'tok/step', round(d['value']*d['ms_per_step']/1e3), d['ppo_phase_s_per_step'])"
done
