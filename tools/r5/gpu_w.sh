#!/bin/bash
# round 5, GPU call W: non-temporal epilogue stores in the large GEMMs (gemm_exp base vs ntstore)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w
mkdir -p $O
for r in 1 2 3; do
  for v in base ntstore; do
    echo "== $v" >> $O/nt.log
    timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> $O/nt.log 2>&1 || exit 1
  done
done
cat $O/nt.log
