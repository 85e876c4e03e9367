#!/bin/bash
# round 5, GPU call L: batch-1 sampler phase timing (tools/sampler_exp) + the sampler GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k sampler --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for S in 1.3 4.0; do
for v in full p2 pA pB p3; do
  for w in 1 0; do
    echo -n "$v " >> $O/phases.log
    timeout -k 10 60 tools/sampler_exp/bin/sampler_exp_$v $([ $v = full ] && echo $w || echo $((w + 100))) $S >> $O/phases.log 2>&1 || { cat $O/phases.log; exit 1; }
  done
done
done
cat $O/phases.log
