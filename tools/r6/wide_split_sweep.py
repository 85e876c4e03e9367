#!/usr/bin/env python3
"""Split-K of the wide M <= 64 decode kernel over bf16 weights (tuning wide_split): time of the
kernel + its reduce launch per split, qkv / o / down at M = 32 and 64, cold weights (4 copies).
Usage (GPU box): python tools/r6/wide_split_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def timeit(fn, n=20, reps=7):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return sorted(ts)[reps // 2]


def main():
    C = ops.native()
    dev = torch.device("cuda")
    for M in (32, 64):
        x = torch.randn(M, 14336, device=dev).to(torch.bfloat16)
        for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336)):
            ws = [(torch.randn(N, K, device=dev) / 64).to(torch.bfloat16) for _ in range(4)]
            xk = x[:, :K].contiguous()
            row = []
            for sp in (0, 2, 4, 8, 16, 32):
                C.set_tuning({"wide_split": sp})
                C.gemm(xk, ws[0], None, None, None, 0, False, None)
                row.append(f"{sp or 'auto'}: {timeit(lambda i: C.gemm(xk, ws[i % 4], None, None, None, 0, False, None)):5.1f}")
            C.set_tuning({"wide_split": 0})
            print(f"M={M} {name:5s} N={N} K={K}: " + " | ".join(row) + " us", flush=True)
            del ws


if __name__ == "__main__":
    main()
