#!/bin/bash
# Build tools/gemm_exp: one standalone timing binary per experiment variant of gemm_big.hip
# (tools/gemm_exp/make_variants.py). CPU-side only (hipcc cross-compiles gfx950); run the binaries
# on the GPU box: for b in tools/gemm_exp/bin/gemm_exp_*; do timeout -k 10 120 $b 10; done
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/gemm_exp/bin
SRC=tools/gemm_exp/src
mkdir -p "$OUT" "$SRC"
python3 tools/gemm_exp/make_variants.py "$SRC" > /dev/null
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -Icsrc/include -Wno-unused-result"
$HIPCC $FLAGS -c tools/gemm_exp/main.cpp -o "$SRC/main.o" &
$HIPCC -O2 -std=c++17 -Icsrc/include -c csrc/host/tuning.cpp -o "$SRC/tuning.o" &
wait
pids=()
for f in "$SRC"/gemm_big_*.hip; do
  v=$(basename "$f" .hip); v=${v#gemm_big_}
  ( $HIPCC $FLAGS -c "$f" -o "$SRC/$v.o" && $HIPCC --offload-arch=gfx950 "$SRC/$v.o" "$SRC/main.o" "$SRC/tuning.o" -o "$OUT/gemm_exp_$v" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls "$OUT"
