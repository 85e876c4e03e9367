#!/bin/bash
# round 4, GPU call C: config 5 (Llama-2-13B RAG -> LoRA SFT -> PPO, fp8 inference / fp8 KV /
# fp8 frozen-base training forwards) at 64 / 128 / 256 rollouts per GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
for rb in ${BATCHES:-64 128 256}; do
  mb=$(( rb >= 256 ? 32 : 16 ))
  timeout -k 10 420 python -u bench.py --mode pipeline --rollout-batch $rb --minibatch $mb --steps 2 --warmup 1 \
    > gpurun_out/r4/c_pipeline13b_rb${rb}.log 2>&1 || { echo "pipeline rb=$rb failed"; tail -20 gpurun_out/r4/c_pipeline13b_rb${rb}.log; exit 1; }
  python3 - "$rb" <<'PY'
import json, sys
rb = sys.argv[1]
line = [l for l in open(f"gpurun_out/r4/c_pipeline13b_rb{rb}.log") if l.startswith("{")][-1]
r = json.loads(line)
print(f"rb={rb} tok/s={r['value']:.0f} ms/step={r['ms_per_step']:.0f} phases={r['ppo_phase_s_per_step']} sft={r['sft']['value']:.0f}")
PY
done
