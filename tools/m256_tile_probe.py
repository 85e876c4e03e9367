"""Batch-256 decode GEMM shapes: the 256x128 gemm_big tile (production) vs the 128x128 two-workgroups-
per-CU tile kernel (gemm_bf16.hip gemm_tile_kernel) and gemm_256_kernel, cold weights (8 rotating
copies > the 256 MB Infinity Cache), hipEvent timing over 40 launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rag_tl_domainllm_optimizer_amd import ops
from rag_tl_domainllm_optimizer_amd.ops.linear import ROW

C = ops.native()
M = 256
x = torch.randn(M, 4096, device="cuda", dtype=torch.bfloat16)
for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
    xs = x if K == 4096 else torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(max(2, 2048 * 2 ** 20 // (N * K * 2) + 1))]
    res = {}
    variants = {
        "big128": lambda w: ops.gemm_big(xs, w, ROW, ROW, bn=128),
        "big_auto": lambda w: ops.gemm(xs, w),
        "tile128": lambda w: (C.set_tuning({"gemm_variant": 1}), C.gemm(xs, w, None, None, None, 0, False, None))[1],
        "k256": lambda w: (C.set_tuning({"gemm_variant": 2}), C.gemm(xs, w, None, None, None, 0, False, None))[1],
    }
    ref = None
    for vname, fn in variants.items():
        for i in range(4):
            y = fn(ws[i % len(ws)])
        torch.cuda.synchronize()
        if ref is None:
            ref = y.float()
        err = (y.float() - ref).abs().max().item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            fn(ws[i % len(ws)])
        e1.record()
        torch.cuda.synchronize()
        C.set_tuning({"gemm_variant": 0})
        res[vname] = (e0.elapsed_time(e1) / 40 * 1e3, err)
    print(f"M=256 {name:8s} N={N:6d} K={K:6d}: " + "  ".join(f"{k}={v[0]:7.1f}us(err {v[1]:.2g})" for k, v in res.items()), flush=True)
    del ws
