#!/bin/bash
# PMC counters for the flash attention kernels (own run: --pmc with kernel trace only)
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/attn_pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "attn_" -f csv -d /tmp/apmc -o run -- python3 $R/tools/attn_probe.py --iters 2 > $R/gpurun_out/attn_pmc/log.txt 2>&1 || exit $?
find /tmp/apmc -name "*counter_collection.csv" -exec cp {} $R/gpurun_out/attn_pmc/ \;
rm -rf /tmp/apmc
