#!/bin/bash
# PMC passes for the batch-256 decode attention kernels (the MFMA kernel; the VALU form is only the
# fallback for head_dim != 128 since round 5)
set -o pipefail
R=$PWD
out=$R/gpurun_out/pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 cnt=$2; shift 2
  rm -rf /tmp/pmca_$name
  timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-include-regex "attn_decode" -f csv -d /tmp/pmca_$name -o run \
    -- python3 $R/tools/decode_attn_probe.py --iters 5 > $out/log_attn_$name.txt 2>&1 || return $?
  find /tmp/pmca_$name -name "*counter_collection.csv" -exec cp {} $out/attn_$name.csv \;
  rm -rf /tmp/pmca_$name
}
run a "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" &&
run f "FETCH_SIZE GRBM_GUI_ACTIVE" &&
run w "WRITE_SIZE"
