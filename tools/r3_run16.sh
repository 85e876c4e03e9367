#!/bin/bash
# wide W8A16 kernel with the in-launch split-K hand-off: numerics, per-shape A/B vs the reduce
# launch, and the 13B batch-64 fp8 decode step.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r3
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "fp8 or swiglu_pair or gemm_decode" > gpurun_out/r3/test_wide_ticket.log 2>&1 || { tail -40 gpurun_out/r3/test_wide_ticket.log; exit 1; }
tail -1 gpurun_out/r3/test_wide_ticket.log
for t in 0 1; do
  RT_WIDE_TICKET=$t timeout -k 10 300 python3 -u tools/fp8_decode_table.py --ms 32,64 > gpurun_out/r3/fp8_table_ticket$t.log 2>&1 || { tail gpurun_out/r3/fp8_table_ticket$t.log; exit 1; }
  echo "== RT_WIDE_TICKET=$t"; grep "^|" gpurun_out/r3/fp8_table_ticket$t.log
done
for t in 0 1; do
  RT_WIDE_TICKET=$t timeout -k 10 300 python3 -u tools/decode_profile.py --model llama2-13b --fp8 --fp8-kv --batch 64 --prompt 320 --new 64 > gpurun_out/r3/dec13b_ticket$t.log 2>&1 || { tail gpurun_out/r3/dec13b_ticket$t.log; exit 1; }
  echo "== RT_WIDE_TICKET=$t"; grep "iter 2" gpurun_out/r3/dec13b_ticket$t.log
done
