#!/usr/bin/env python3
"""Decode GEMMs at 16 < M <= 64 (serving / small rollout batches): the 64-column LDS-DMA ring
(gemm_m64_kernel, tuning m64_wide = 0), the 256-row wide kernel over row-major weights
(m64_wide = 1) and, for qkv / o, the 256x128 split-K gemm_big form ops.gemm picks at 32 <= M <= 64.
Mistral-7B shapes, cold weights (4 copies, round robin), median of 7 x 20 launches; us per call.
Usage (GPU box): python tools/r6/m64_wide_probe.py"""
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
    ts.sort()
    return ts[reps // 2]


def main():
    C = ops.native()
    dev = torch.device("cuda")
    shapes = [("qkv", 6144, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, ops.ACT_SWIGLU),
              ("down", 4096, 14336, 0), ("lm_head", 32000, 4096, 0)]
    for M in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "24,32,48,64").split(",")]:
        x = torch.randn(M, 14336, device=dev).to(torch.bfloat16)
        tot = {"ring": 0.0, "wide": 0.0, "ops.gemm": 0.0}
        for name, N, K, act in shapes:
            ws = [(torch.randn(N, K, device=dev) / 64).to(torch.bfloat16) for _ in range(4)]
            xk = x[:, :K].contiguous()
            res = {}
            for mode, wide in (("ring", 0), ("wide", 1)):
                C.set_tuning({"m64_wide": wide})
                C.gemm(xk, ws[0], None, None, None, act, False, None)
                res[mode] = timeit(lambda i: C.gemm(xk, ws[i % 4], None, None, None, act, False, None))
            C.set_tuning({"m64_wide": 1})
            res["ops.gemm"] = timeit(lambda i: ops.gemm(xk, ws[i % 4], act=act))
            y0 = C.gemm(xk, ws[0], None, None, None, act, False, None).float()
            C.set_tuning({"m64_wide": 0})
            y1 = C.gemm(xk, ws[0], None, None, None, act, False, None).float()
            C.set_tuning({"m64_wide": 1})
            err = float((y0 - y1).abs().max() / y1.abs().max().clamp(min=1e-6))
            for k in tot:
                tot[k] += res[k]
            mb = N * K * 2 / 1e6
            print(f"M={M:2d} {name:8s} N={N:5d} K={K:5d}: ring {res['ring']:6.1f} us ({mb / res['ring']:.2f} TB/s) | "
                  f"wide {res['wide']:6.1f} us ({mb / res['wide']:.2f} TB/s) | ops.gemm {res['ops.gemm']:6.1f} us | "
                  f"wide vs ring rel diff {err:.1e}", flush=True)
            del ws
        print(f"M={M:2d} layer total: ring {tot['ring']:.1f} us, wide {tot['wide']:.1f} us, ops.gemm dispatch "
              f"{tot['ops.gemm']:.1f} us", flush=True)


if __name__ == "__main__":
    main()
