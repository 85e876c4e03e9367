#!/bin/bash
# Round-6 call AS: heaviest-first (LPT) dispatch order of the causal attention grids — bitwise /
# oracle tests of every attention form, then the timing A/B at the PPO shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/as
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" \
  > gpurun_out/as/tests.log 2>&1 || { tail -30 gpurun_out/as/tests.log; exit 1; }
tail -2 gpurun_out/as/tests.log
timeout -k 10 300 python -u tools/r6/attn_lpt_probe.py --rounds 5 > gpurun_out/as/probe.log 2>&1
rc=$?; cat gpurun_out/as/probe.log | tail -8; exit $rc
