#!/bin/bash
# Build tools/gemm_exp/run/gemm_m256_pad{,_xonly,_wonly}: gemm_big's batch-256 forms at padded /
# unpadded operand strides (m256_pad_main.cpp), linked with gemm_m256ws.hip streaming both operands,
# only the activations (GM_EXP=3) or only the weights (GM_EXP=4). Run on the GPU box.
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/gemm_exp/run
SRC=tools/gemm_exp/src
mkdir -p "$OUT" "$SRC"
H=/opt/rocm/bin/hipcc
F="-O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -Icsrc/include -Wno-unused-result"
$H $F -c csrc/kernels/gemm_big.hip -o $SRC/gb.o &
$H $F -c tools/gemm_exp/m256_pad_main.cpp -o $SRC/m256_pad_main.o &
$H -O2 -std=c++17 -Icsrc/include -c csrc/host/tuning.cpp -o $SRC/tuning.o &
$H $F -c tools/gemm_exp/gemm_m256ws.hip -o $SRC/ws_both.o &
$H $F -DGM_EXP=3 -c tools/gemm_exp/gemm_m256ws.hip -o $SRC/ws_xonly.o &
$H $F -DGM_EXP=4 -c tools/gemm_exp/gemm_m256ws.hip -o $SRC/ws_wonly.o &
wait
for v in both xonly wonly; do
  $H --offload-arch=gfx950 $SRC/ws_$v.o $SRC/gb.o $SRC/m256_pad_main.o $SRC/tuning.o -o $OUT/gemm_m256_pad_$v
done
ls $OUT
