#!/bin/bash
# PMC comparison on the qkv update shape: 8-wave gemm_big (nt), 4-wave tiles (w4_256, w4_192), hipBLASLt (lib_nt).
set -o pipefail
R=$PWD
out=$R/gpurun_out/w4_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {  # $1 tag, rest counters
  tag=$1; shift
  rm -rf /tmp/w4p
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "gemm_big|gemm_w4|Cijk" -f csv -d /tmp/w4p -o run -- \
    python3 $R/tools/gemm_big_probe.py --M 9632 --shapes qkv --cases nt,w4_256,w4_192,lib_nt --rounds 1 --iters 3 > $out/log_$tag.txt 2>&1 || return 1
  find /tmp/w4p -name "*counter_collection.csv" -exec cp {} $out/pmc_$tag.csv \;
  python3 $R/tools/pmc_summary.py $out/pmc_$tag.csv > $out/summary_$tag.txt 2>&1
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
run b SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES && \
cat $out/summary_a.txt $out/summary_b.txt
