#!/bin/bash
# round 5, GPU call G: B-direct NT GEMM experiment (tools/gemm_exp/gemm_bdirect.hip) vs gemm_big;
# bd_exp_hot re-reads the first K-step's fragments every step (issue cost without L2 misses)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
for b in bd_exp bd_exp_hot bd_exp; do
  echo "== $b" >> $O/bd2.log
  timeout -k 10 120 tools/gemm_exp/bin/$b 10 >> $O/bd2.log 2>&1 || { cat $O/bd2.log; exit 1; }
done
cat $O/bd2.log
