#!/bin/bash
# round 4, GPU call B: full GPU test tier (tuning / side-channel refactor), then a phase-synced PPO profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/r4/b_gpu_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/r4/b_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r4/b_gpu_tests.log
PROF_TAG=b_prof_ppo bash tools/r4/prof_ppo.sh
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u tools/gemm_big_probe.py --M 9632 --cases nt,nn,lib_nt --sweep gemm_group_m=2,8,16 --rounds 3 \
  > gpurun_out/r4/b_group_m_sweep.log 2>&1 && grep -v amdgpu.ids gpurun_out/r4/b_group_m_sweep.log
