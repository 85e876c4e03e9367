#!/bin/bash
# Build tools/gemm_exp/run/gemm_m256_exp{,_x1,_x2}: the one-section batch-256 decode GEMM
# (gemm_m256.hip; _x1 without MFMAs, _x2 without LDS-DMA after the prologue) against gemm_big.
# CPU-side only; run on the GPU box: timeout -k 10 60 tools/gemm_exp/run/gemm_m256_exp 256
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/gemm_exp/run
SRC=tools/gemm_exp/src
mkdir -p "$OUT" "$SRC"
H=/opt/rocm/bin/hipcc
F="-O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -Icsrc/include -Wno-unused-result"
$H $F -c csrc/kernels/gemm_big.hip -o $SRC/gb.o &
$H $F -c tools/gemm_exp/m256_main.cpp -o $SRC/m256_main.o &
$H -O2 -std=c++17 -Icsrc/include -c csrc/host/tuning.cpp -o $SRC/tuning.o &
$H $F -c tools/gemm_exp/gemm_m256.hip -o $SRC/m256.o &
$H $F -DGM_EXP=1 -c tools/gemm_exp/gemm_m256.hip -o $SRC/m256_x1.o &
$H $F -DGM_EXP=2 -c tools/gemm_exp/gemm_m256.hip -o $SRC/m256_x2.o &
wait
for v in "" _x1 _x2; do
  $H --offload-arch=gfx950 $SRC/m256$v.o $SRC/gb.o $SRC/m256_main.o $SRC/tuning.o -o $OUT/gemm_m256_exp$v
done
ls $OUT
