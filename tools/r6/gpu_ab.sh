#!/bin/bash
# Round-6 call AB: 4-wave decode attention for 256 <= batch x kv heads < 1024 (serving batch 32..127)
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "decode" > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || exit $rc
for b in 32 48 64 96; do
  for bh in 256 1024; do
    echo "batch $b decode_mw_bh $bh" | tee -a gpurun_out/ab/steps.log
    timeout -k 10 300 python3 -u tools/decode_profile.py --batch $b --prompt 173 --new 64 --iters 2 --set decode_mw_bh=$bh 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a gpurun_out/ab/steps.log || exit 1
  done
done
