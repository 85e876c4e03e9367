#!/bin/bash
# round 4, GPU call A: stream-K + tuning refactor correctness, then GEMM probe (SK on / off / lib)
set -o pipefail
mkdir -p gpurun_out/r4
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gemm_big_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4/a_gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/r4/a_gemm_tests.log; exit 1; }
tail -3 gpurun_out/r4/a_gemm_tests.log
timeout -k 10 400 python -u tools/gemm_big_probe.py --M 9632 19264 \
  --cases nt,nt_nosk,lib_nt,nn,nn_nosk,lib_nn,nt_swiglu,nt_swiglu_nosk --rounds 3 > gpurun_out/r4/a_gemm_probe.log 2>&1
rc=$?
cat gpurun_out/r4/a_gemm_probe.log | grep -v amdgpu.ids
exit $rc
