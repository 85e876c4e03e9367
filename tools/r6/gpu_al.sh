#!/bin/bash
# Round-6 call AL: token-parallel GEMMs vs hipBLASLt (comparator only), same box, final tree
set -o pipefail
mkdir -p gpurun_out/al
timeout -k 10 600 python -u tools/gemm_big_probe.py --M 9632 --rounds 5 --cases nt,lib_nt,nn,lib_nn,nt_swiglu 2>&1 | grep -v amdgpu.ids | tee gpurun_out/al/gemm_probe.log
