#!/bin/bash
# round 4, GPU call J: same-box A/B of the headline bench, tree of call E (0d31371, _ab_old/e) vs the
# current tree, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
for r in old new old new; do
  if [ $r = old ]; then d=_ab_old/e; else d=.; fi
  ( cd $d && timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 ) > gpurun_out/r4/j_bench_$r.log.$$ 2>&1 || { echo "bench $r failed"; tail -20 gpurun_out/r4/j_bench_$r.log.$$; exit 1; }
  cat gpurun_out/r4/j_bench_$r.log.$$ >> gpurun_out/r4/j_bench_$r.log; rm -f gpurun_out/r4/j_bench_$r.log.$$
  grep '^{' gpurun_out/r4/j_bench_$r.log | tail -1 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('bench $r', round(r['value']), round(r['ms_per_step']), r['p50_rag_latency_s'], r['phase_s_per_step'])"
done
