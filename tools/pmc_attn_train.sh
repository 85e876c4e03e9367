#!/bin/bash
# PMC passes for the training flash-attention kernels (tools/attn_train_probe.py)
set -o pipefail
R=$PWD
out=$R/gpurun_out/pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 cnt=$2; shift 2
  rm -rf /tmp/pmct_$name
  timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-include-regex "attn_" -f csv -d /tmp/pmct_$name -o run \
    -- python3 $R/tools/attn_train_probe.py --iters 3 > $out/log_attntr_$name.txt 2>&1 || return $?
  find /tmp/pmct_$name -name "*counter_collection.csv" -exec cp {} $out/attntr_$name.csv \;
  rm -rf /tmp/pmct_$name
}
run a "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" &&
run f "FETCH_SIZE GRBM_GUI_ACTIVE"
