#!/bin/bash
# round 5, GPU call F: ceiling of a GEMM whose B operand bypasses LDS (tools/gemm_exp variants
# base / nob (no B LDS traffic, constant B) / bglb (B rows straight from global into VGPRs))
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5f
mkdir -p $O
for r in 1 2; do
  for v in base nob bglb; do
    echo "== $v" >> $O/bbypass.log
    timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> $O/bbypass.log 2>&1 || exit 1
  done
done
cat $O/bbypass.log
