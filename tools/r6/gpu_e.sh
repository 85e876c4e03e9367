# round 6 call E: same-box A/B of the LoRA gradient epilogue (off / on / off / on)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for m in off on; do
    timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --skip-latency --lora-grad-epilogue $m > gpurun_out/b_lge_${m}_$i.log 2>&1 || exit 1
    echo "$m $i $(grep -o '"value": [0-9.]*' gpurun_out/b_lge_${m}_$i.log) $(grep -o '"time/update": [0-9.]*' gpurun_out/b_lge_${m}_$i.log)"
  done
done
