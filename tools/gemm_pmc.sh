#!/bin/bash
# PMC counters of the token-parallel GEMMs (own runs: --pmc with kernel trace only, one pass each)
# Usage (GPU box, repo root): tools/gemm_pmc.sh <probe args...>
set -o pipefail
R=$PWD
out=$R/gpurun_out/gemm_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  local cnt=$1; shift
  rm -rf /tmp/gpmc_$name
  timeout -s KILL 120 rocprofv3 --pmc $cnt --kernel-include-regex "gemm_big|Cijk|gemm_256" -f csv -d /tmp/gpmc_$name -o run \
    -- python3 $R/tools/gemm_big_probe.py "$@" > $out/log_$name.txt 2>&1 || return $?
  find /tmp/gpmc_$name -name "*counter_collection.csv" -exec cp {} $out/$name.csv \;
  rm -rf /tmp/gpmc_$name
}
pass sq "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE" "$@" &&
pass tcc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA" "$@"
