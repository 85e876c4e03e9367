"""Narrow LoRA products on the 64x64 vs 128x64 tiles of gemm_small_kernel, kernel only (outputs
pre-zeroed outside the timed loop), PPO-update token count, the split counts ops.linear picks.

    python tools/small_bm_probe.py [--M 9632]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=9632)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    C = ops.native()
    dev, M, R = "cuda", a.M, 64
    for K in (4096, 6144, 14336, 28672):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ap_ = (torch.randn(R, K, device=dev) / 64).to(torch.bfloat16)
        ub = (torch.randn(K, R, device=dev) / 64).to(torch.bfloat16)
        du = torch.randn(M, R, device=dev).to(torch.bfloat16)
        o_mr = torch.zeros(M, R, device=dev)
        o_kr = torch.zeros(K, R, device=dev)
        o_rk = torch.zeros(R, K, device=dev)
        tiles = lambda P, Q, bm: ((P + bm - 1) // bm) * ((Q + 63) // 64)  # noqa: E731
        cases = {}
        for bm in (64, 128):
            ns_u = 1 if K <= 4096 else max(1, min(K // 512, (768 + tiles(M, R, bm) - 1) // tiles(M, R, bm)))
            ns_tn_b = max(1, min(M // 256, (1024 + tiles(K, R, bm) - 1) // tiles(K, R, bm)))
            ns_tn_a = max(1, min(M // 256, (1024 + tiles(R, K, bm) - 1) // tiles(R, K, bm)))
            cases[f"u{bm}"] = (lambda bm=bm, ns=ns_u: C.gemm_small(x, ap_, 0, 0, 2, ns, o_mr, bm)) if ns_u > 1 else \
                (lambda bm=bm: C.gemm_small(x, ap_, 0, 0, 0, 1, None, bm))
            cases[f"du{bm}"] = lambda bm=bm, ns=ns_u: C.gemm_small(x, ub, 0, 1, 2, max(ns, 1), o_mr, bm)
            cases[f"dB{bm}"] = lambda bm=bm, ns=ns_tn_b: C.gemm_small(x, du, 1, 1, 2, ns, o_kr, bm)
            cases[f"dA{bm}"] = lambda bm=bm, ns=ns_tn_a: C.gemm_small(du, x, 1, 1, 2, ns, o_rk, bm)
        res = {k: [] for k in cases}
        for _ in range(a.rounds):
            for k, fn in cases.items():
                res[k].append(timeit(fn))
        gb = M * K * 2 / 1e9
        print(f"M={M} K={K}: " + " ".join(f"{k}={statistics.median(v):7.1f}us({gb / statistics.median(v) * 1e3:4.2f}TB/s)"
                                         for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
