#!/bin/bash
# PMC passes for the batch-1 RAG-answer decode loop (Mistral-7B + LoRA r16, prompt 173): bytes moved
# by the weight-streaming GEMVs (gemv16_kernel, tile-ordered weights, no split-K) and the fused decode
# attention (8-wave attn_decode_mfma_kernel). One counter group per run, kernel trace only.
# Usage (GPU box, repo root): tools/pmc_decode_b1.sh ; summary: python tools/pmc_summary.py gpurun_out/pmc_b1/*.csv
set -o pipefail
R=$PWD
out=$R/gpurun_out/pmc_b1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 cnt=$2
  rm -rf /tmp/pmcb1_$name
  timeout -s KILL 150 rocprofv3 --pmc $cnt --kernel-include-regex "gemm_decode|gemv16|attn_decode" -f csv \
    -d /tmp/pmcb1_$name -o run -- python3 $R/tools/decode_profile.py --batch 1 --prompt 173 --new 16 \
    > $out/log_$name.txt 2>&1 || return $?
  find /tmp/pmcb1_$name -name "*counter_collection.csv" -exec cp {} $out/b1_$name.csv \;
  rm -rf /tmp/pmcb1_$name
}
run f "FETCH_SIZE GRBM_GUI_ACTIVE" &&
run w "WRITE_SIZE" &&
run a "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE"
