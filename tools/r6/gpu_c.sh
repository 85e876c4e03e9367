# round 6 call C: K-rotation probe for the batch-256 decode GEMMs; per-layer divergence trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6/m256_krot_probe.py > gpurun_out/krot_probe.log 2>&1 || exit 1
cat gpurun_out/krot_probe.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/r6/divergence_trace.py --batch 1 --steps 24 > gpurun_out/div_b1.log 2>&1 || exit 1
cat gpurun_out/div_b1.log | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/r6/divergence_trace.py --batch 256 --steps 12 --oracle-rows 2 > gpurun_out/div_b256.log 2>&1 || exit 1
cat gpurun_out/div_b256.log | grep -v amdgpu.ids
timeout -k 10 120 ./tools/r6/mfma_probe > gpurun_out/mfma_probe2.log 2>&1 || exit 1
cat gpurun_out/mfma_probe2.log
