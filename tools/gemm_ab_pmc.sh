#!/bin/bash
# Ours vs hipBLASLt on the PPO-update NT shapes (M = 9632): wall time (probe, no profiler) and one
# PMC pass of matrix-core busy / wave counters per kernel (kernel trace only, one group).
# Usage (GPU box, repo root): bash tools/gemm_ab_pmc.sh
set -o pipefail
R=$PWD
out=$R/gpurun_out/gemm_ab
mkdir -p $out
timeout -k 10 300 python3 $R/tools/gemm_big_probe.py --M 9632 --shapes qkv,gate_up --cases nt,lib_nt,auto --rounds 5 \
  > $out/timing.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/gab
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  --kernel-include-regex "gemm_big|Cijk" -f csv -d /tmp/gab -o run -- python3 $R/tools/gemm_big_probe.py --M 9632 \
  --shapes qkv,gate_up --cases nt,lib_nt --rounds 1 --iters 3 > $out/pmc_log.txt 2>&1 || exit $?
find /tmp/gab -name "*counter_collection.csv" -exec cp {} $out/pmc.csv \;
rm -rf /tmp/gab
python3 $R/tools/pmc_summary.py $out/pmc.csv > $out/pmc_summary.txt 2>&1
cat $out/timing.log $out/pmc_summary.txt
