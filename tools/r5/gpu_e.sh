#!/bin/bash
# round 5, GPU call E: cost of the bf16 epilogue inside the large GEMMs (tools/gemm_exp variants
# base / nostore / noepi, interleaved twice on one box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5e
mkdir -p $O
for r in 1 2; do
  for v in base nostore noepi; do
    echo "== $v" >> $O/epi.log
    timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> $O/epi.log 2>&1 || exit 1
  done
done
cat $O/epi.log
