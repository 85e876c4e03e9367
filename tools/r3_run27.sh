#!/bin/bash
# config 5 pipeline with the SFT stage's frozen-base forwards on W8A8 too.
set -o pipefail
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u bench.py --mode pipeline --steps 2 --warmup 1 > gpurun_out/r3/bench_pipeline_fp8sft.log 2>&1 || { tail -30 gpurun_out/r3/bench_pipeline_fp8sft.log; exit 1; }
grep "sft warmup" gpurun_out/r3/bench_pipeline_fp8sft.log; tail -1 gpurun_out/r3/bench_pipeline_fp8sft.log
