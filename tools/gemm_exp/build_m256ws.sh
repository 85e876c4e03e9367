#!/bin/bash
# Build tools/gemm_exp/run/gemm_m256ws_x{XS}w{WS}n{NT}: the wave-specialised batch-256 decode GEMM
# (gemm_m256ws.hip) against gemm_big, one binary per (activation stages, weight stages, nt) variant.
# CPU-side only; run on the GPU box: timeout -k 10 60 tools/gemm_exp/run/gemm_m256ws_x3w4n0 256
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
VARIANTS="3:4:0 3:4:1 2:6:0 2:6:1"
for v in $VARIANTS; do
  IFS=: read xs ws nt <<<"$v"
  $H $F -DGM_XS=$xs -DGM_WS=$ws -DGM_NT=$nt -c tools/gemm_exp/gemm_m256ws.hip -o $SRC/m256ws_x${xs}w${ws}n${nt}.o &
done
wait
for v in $VARIANTS; do
  IFS=: read xs ws nt <<<"$v"
  $H --offload-arch=gfx950 $SRC/m256ws_x${xs}w${ws}n${nt}.o $SRC/gb.o $SRC/m256_main.o $SRC/tuning.o \
    -o $OUT/gemm_m256ws_x${xs}w${ws}n${nt}
done
ls $OUT
