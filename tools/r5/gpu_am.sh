#!/bin/bash
# round 5, GPU call AM: LoRA narrow-product splits — GPU tests, then PPO step A/B (new rules vs previous ops/linear.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_big_gpu.py \
  -k "lora or narrow or small or tn" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
L=rag_tl_domainllm_optimizer_amd/ops/linear.py
cp $L /tmp/linear_new.py
for r in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then cp /tmp/linear_new.py $L; else cp tools/r5/linear_prev.py.txt $L; fi
    echo "== $v" >> $O/bench.log
    timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 --skip-latency >> $O/bench.log 2>&1 || { cp /tmp/linear_new.py $L; tail -20 $O/bench.log; exit 1; }
  done
done
cp /tmp/linear_new.py $L
grep -E "^==|^\{" $O/bench.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip(), end=' ')
    else:
        d = json.loads(l); print(round(d['value'], 1), round(d['ms_per_step'], 1), {k: round(v, 3) for k, v in d['phase_s_per_step'].items()})"
