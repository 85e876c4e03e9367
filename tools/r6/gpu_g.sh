# round 6 call G: secondary modes on the round-6 tree (config 3 SFT, config 5 pipeline, full-FT PPO,
# serving) and a 2-rank data-parallel rehearsal on one GPU over gloo (GradSync overlap hooks incl.
# the LoRA epilogue's direct-gradient readiness signal; not a scaling point)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --mode sft --steps 3 --warmup 1 > gpurun_out/g_sft.log 2>&1 || exit 1
tail -1 gpurun_out/g_sft.log | cut -c1-300
timeout -k 10 900 python -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/g_pipe.log 2>&1 || exit 1
tail -1 gpurun_out/g_pipe.log | cut -c1-300
timeout -k 10 900 python -u bench.py --full-ft --steps 2 --warmup 1 --skip-latency > gpurun_out/g_fullft.log 2>&1 || exit 1
tail -1 gpurun_out/g_fullft.log | cut -c1-300
RAGTL_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 2 --warmup 1 --skip-latency --rollout-batch 64 > gpurun_out/g_dp2_gloo.log 2>&1 || exit 1
tail -1 gpurun_out/g_dp2_gloo.log | cut -c1-400
