#!/bin/bash
# round 4, GPU call F: which stall bounds the 256x256 GEMM (tools/gemm_exp variants; timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
for v in base nowait nobar_end noprio nolgkm nowait_nobar_end base; do
  echo "== $v" >> gpurun_out/r4/f_gemm_exp.log
  timeout -k 10 120 tools/gemm_exp/bin/gemm_exp_$v 10 >> gpurun_out/r4/f_gemm_exp.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r4/f_gemm_exp.log; exit 1; }
done
cat gpurun_out/r4/f_gemm_exp.log
