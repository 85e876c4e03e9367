#!/usr/bin/env python3
"""Residual-add + RMSNorm forward at the update's shape (9632 x 4096 bf16: reads x, residual; writes y,
h = 316 MB) against torch's own streaming kernels of similar byte counts, to tell whether the norm is
at the chip's read+write rate. Usage (GPU box): python tools/r6/norm_bw_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return sorted(ts)[2]


def main():
    T, H = 9632, 4096
    dev = torch.device("cuda")
    xs = [torch.randn(T, H, device=dev).to(torch.bfloat16) for _ in range(4)]
    rs = [torch.randn(T, H, device=dev).to(torch.bfloat16) for _ in range(4)]
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    C = ops.native()
    mb = T * H * 2 / 1e6
    it = [0]

    def norm():
        i = it[0] = (it[0] + 1) % 4
        C.norm_fwd(False, xs[i], rs[i], w, None, 1e-5)

    def add():
        i = it[0] = (it[0] + 1) % 4
        torch.add(xs[i], rs[i])

    def copy():
        i = it[0] = (it[0] + 1) % 4
        xs[i].clone()

    for name, fn, nbytes in (("norm_fwd (x + res -> y, h)", norm, 4 * mb), ("torch add (2 reads, 1 write)", add, 3 * mb),
                             ("torch clone (1 read, 1 write)", copy, 2 * mb)):
        t = timeit(fn)
        print(f"{name:32s} {t:7.1f} us  {nbytes / t:.2f} TB/s of read + write bytes", flush=True)


if __name__ == "__main__":
    main()
