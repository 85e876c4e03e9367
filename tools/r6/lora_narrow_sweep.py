#!/usr/bin/env python3
"""LoRA backward narrow products after the move to fixed-order slabs (round 6): split sweeps of
dU = dY UB (ops.linear._narrow, KMAJ adapter image, slabs + splitk_reduce) and of the token-split
TN products dA = dU^T X / dB = dY^T U (ops.linear._tn_slabs, summed here by a torch reduction as
lora_grad_accum would), at the update's 9632 tokens; us per call, median of 7 x 10, rotating inputs.
Usage (GPU box): python tools/r6/lora_narrow_sweep.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
L = importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear")


def timeit(fn, n=10, reps=7):
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
    dev = torch.device("cuda")
    T = 9632
    C = L.native()
    for name, N in (("qkv", 6144), ("o", 4096), ("gate_up", 28672), ("down", 4096)):
        dys = [torch.randn(T, N, device=dev).to(torch.bfloat16) for _ in range(2)]
        ub = (torch.randn(N, 64, device=dev) / 64).to(torch.bfloat16)
        row = []
        for ns in (0, 4, 6, 8, 11, 16, 24):
            row.append(f"{ns or 'auto'}: {timeit(lambda i: L._narrow(dys[i % 2], ub, L.KMAJ, ns)):6.1f}")
        print(f"dU {name:8s} N={N:5d}: " + " | ".join(row), flush=True)
        u = torch.randn(T, 64, device=dev).to(torch.bfloat16)
        row = []
        for ns in (2, 4, 8, 12, 16):
            P, Q = N, 64
            bm = 128 if P >= 16384 else 64

            def fn(i, ns=ns, bm=bm):
                ws = torch.empty(ns * P * Q, dtype=torch.float32, device=dev).view(ns * P, Q)
                C.gemm_small(dys[i % 2], u, L.KMAJ, L.KMAJ, 3, ns, ws, bm)
            row.append(f"{ns}: {timeit(fn):6.1f}")
        print(f"dB {name:8s} N={N:5d}: " + " | ".join(row) + "   (auto = gemm_tn's plan)", flush=True)
        del dys
    # dA = dU^T X [64, K] (K = 4096: qkv / o / gate_up inputs; 14336: down's input)
    for K in (4096, 14336):
        xs = [torch.randn(T, K, device=dev).to(torch.bfloat16) for _ in range(2)]
        du = torch.randn(T, 64, device=dev).to(torch.bfloat16)
        row = []
        for ns in (2, 4, 8, 12, 16):
            def fn(i, ns=ns):
                ws = torch.empty(ns * 64 * K, dtype=torch.float32, device=dev).view(ns * 64, K)
                C.gemm_small(du, xs[i % 2], L.KMAJ, L.KMAJ, 3, ns, ws, 64)
            row.append(f"{ns}: {timeit(fn):6.1f}")
        print(f"dA K={K:5d}: " + " | ".join(row), flush=True)
        del xs


if __name__ == "__main__":
    main()
