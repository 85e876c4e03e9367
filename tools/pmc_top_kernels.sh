#!/bin/bash
# PMC counters for the top kernels of the PPO step, one counter group per run
# (--pmc with kernel trace only; never combined with sys / runtime / marker traces):
#   gemm : the token-parallel GEMM family on the PPO-update shapes (tools/gemm_big_probe.py, M=9632)
#          and the M=256 decode shapes
#   dec  : the batch-256 decode loop (attention + decode GEMMs + split-K reduce), tools/decode_profile.py
# Output: gpurun_out/pmc/<prog>_<pass>.csv ; summarise with tools/pmc_summary.py
set -o pipefail
R=$PWD
out=$R/gpurun_out/pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
run() {  # prog pass counters regex -- cmd...
  local prog=$1 name=$2 cnt=$3 rx=$4; shift 5
  rm -rf /tmp/pmc_$prog$name
  timeout -s KILL 150 rocprofv3 --pmc $cnt --kernel-include-regex "$rx" -f csv -d /tmp/pmc_$prog$name -o run \
    -- "$@" > $out/log_${prog}_$name.txt 2>&1 || return $?
  find /tmp/pmc_$prog$name -name "*counter_collection.csv" -exec cp {} $out/${prog}_$name.csv \;
  rm -rf /tmp/pmc_$prog$name
}
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
G=(python3 $R/tools/gemm_big_probe.py --M 9632 256 --shapes qkv,gate_up,down --cases nt,nn,auto --rounds 1 --iters 2)
D=(python3 $R/tools/decode_profile.py --batch 256 --prompt 173 --new 16)
RX="gemm_big|gemm_small|splitk_reduce|attn_decode"
run gemm a "$A" "$RX" -- "${G[@]}" &&
run gemm f "FETCH_SIZE GRBM_GUI_ACTIVE" "$RX" -- "${G[@]}" &&
run gemm w "WRITE_SIZE" "$RX" -- "${G[@]}" &&
run dec a "$A" "$RX" -- "${D[@]}" &&
run dec f "FETCH_SIZE GRBM_GUI_ACTIVE" "$RX" -- "${D[@]}" &&
run dec w "WRITE_SIZE" "$RX" -- "${D[@]}"
