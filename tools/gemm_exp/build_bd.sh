#!/bin/bash
# Build tools/gemm_exp/bin/bd_exp: the B-direct NT GEMM experiment (gemm_bdirect.hip) against
# gemm_big. CPU-side only; run on the GPU box: timeout -k 10 120 tools/gemm_exp/bin/bd_exp 10
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/gemm_exp/bin
SRC=tools/gemm_exp/src
mkdir -p "$OUT" "$SRC"
H=/opt/rocm/bin/hipcc
F="-O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -Icsrc/include -Wno-unused-result"
$H $F -c csrc/kernels/gemm_big.hip -o $SRC/gb.o &
$H $F -c tools/gemm_exp/bd_main.cpp -o $SRC/bd_main.o &
$H -O2 -std=c++17 -Icsrc/include -c csrc/host/tuning.cpp -o $SRC/tuning.o &
$H $F -c tools/gemm_exp/gemm_bdirect.hip -o $SRC/bd.o &
$H $F -DBD_HOT=1 -c tools/gemm_exp/gemm_bdirect.hip -o $SRC/bd_hot.o &
wait
$H --offload-arch=gfx950 $SRC/bd.o $SRC/gb.o $SRC/bd_main.o $SRC/tuning.o -o $OUT/bd_exp
$H --offload-arch=gfx950 $SRC/bd_hot.o $SRC/gb.o $SRC/bd_main.o $SRC/tuning.o -o $OUT/bd_exp_hot
ls $OUT
