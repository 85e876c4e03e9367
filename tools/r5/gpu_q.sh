#!/bin/bash
# round 5, GPU call Q: fp8 split-K decode + register row quantiser: tests, config-5 pipeline bench + profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "fp8" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u bench.py --mode pipeline --steps 3 --warmup 1 --skip-latency > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 2; }
python3 -c "import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ppo_phase_s_per_step'], 'sft', round(d['sft']['value'],1))"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 3; }
tail -1 $O/tests2.log
