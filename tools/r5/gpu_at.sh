#!/bin/bash
# round 5, GPU call AT: dK/dV backward without the dead K / dS LDS tiles — tests, timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5at
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_props_gpu.py \
  -k "flash or attention" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd tools/r5 && timeout -k 10 300 python -u attn_dq_hp_probe.py > ../../$O/probe.log 2>&1 || { tail -20 ../../$O/probe.log; exit 1; }
cd ../.. && grep us $O/probe.log
