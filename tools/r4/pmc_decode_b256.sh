#!/bin/bash
# Hardware counters of the batch-256 rollout decode loop on the current tree (decode_b256_table.md):
# three --pmc passes with kernel trace only (never combined with other traces), one counter group
# each, over tools/decode_profile.py (Mistral-7B, 256 rows, 173-token prompts, 32 new tokens; eager
# decode steps: counter collection over hipGraph replays crashed the profiler on this image).
# Output: gpurun_out/pmc_b256/{a,f,w}.csv + summary.txt (tools/pmc_summary.py)
set -o pipefail
R=$PWD
out=$R/gpurun_out/pmc_b256
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {  # pass counters
  local name=$1 cnt=$2
  rm -rf /tmp/pmc_b256$name
  timeout -s KILL 170 rocprofv3 --pmc $cnt --kernel-include-regex "gemm_big|norm_fwd|attn_decode|sample" -f csv \
    -d /tmp/pmc_b256$name -o run -- python3 $R/tools/decode_profile.py --batch 256 --prompt 173 --new 32 --iters 1 --no-graph \
    > $out/log_$name.txt 2>&1 || return $?
  find /tmp/pmc_b256$name -name "*counter_collection.csv" -exec cp {} $out/$name.csv \;
  rm -rf /tmp/pmc_b256$name
}
run a "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE" &&
run f "FETCH_SIZE GRBM_GUI_ACTIVE" &&
run w "WRITE_SIZE" &&
python3 $R/tools/pmc_summary.py $out/a.csv $out/f.csv $out/w.csv > $out/summary.txt
