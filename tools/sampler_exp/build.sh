#!/bin/bash
# Build tools/sampler_exp/bin/sampler_exp_{full,p1,p2,p3} (CPU-side only; run on the GPU box)
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/sampler_exp/bin
SRC=tools/sampler_exp/src
mkdir -p "$OUT" "$SRC"
python3 tools/sampler_exp/make_variants.py "$SRC" > /dev/null
H=/opt/rocm/bin/hipcc
F="-O3 --offload-arch=gfx950 -std=c++17 -Icsrc/include -Wno-unused-result"
$H $F -c tools/sampler_exp/main.cpp -o $SRC/main.o &
$H -O2 -std=c++17 -Icsrc/include -c csrc/host/tuning.cpp -o $SRC/tuning.o &
for v in full p1 p2 p3 pA pB; do $H $F -c $SRC/sampling_$v.hip -o $SRC/s_$v.o & done
wait
for v in full p1 p2 p3 pA pB; do $H --offload-arch=gfx950 $SRC/s_$v.o $SRC/main.o $SRC/tuning.o -o $OUT/sampler_exp_$v; done
ls $OUT
