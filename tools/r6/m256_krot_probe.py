"""[round 6, rejected and removed from the kernel: profiles/r6/m256_krot_probe_rejected.log] Batch-256 decode GEMMs with and without the tile-rotated K order (tuning gemm_krot): the split-K
slab forms of qkv / o / down (plan of ops.linear.splitk_plan) and gate_up + SwiGLU, cold weights
(rotating copies > the 256 MB Infinity Cache), hipEvent timing over 40 launches, checksums vs krot 0."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from rag_tl_domainllm_optimizer_amd import ops
from rag_tl_domainllm_optimizer_amd.ops.linear import ACT_SWIGLU, splitk_plan

C = ops.native()
M = 256
for name, N, K, act in (("qkv", 6144, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, ACT_SWIGLU),
                        ("down", 4096, 14336, 0)):
    xs = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
          for _ in range(max(2, 1024 * 2 ** 20 // (N * K * 2) + 1))]
    s, bn = splitk_plan(M, N, K, act)
    slabs = torch.empty(s * M * N, dtype=torch.float32, device="cuda")

    def run(w):
        if act == ACT_SWIGLU:
            return ops.gemm(xs, w, act=ACT_SWIGLU)
        C.gemm_splitk_raw(xs, w, s, slabs, bn or 256)
        return slabs.view(s, M, N).sum(0)

    res = {}
    ref = None
    for kr in (0, 1, 0, 1):
        with ops.tuning(gemm_krot=kr):
            for i in range(4):
                y = run(ws[i % len(ws)])
            torch.cuda.synchronize()
            y = run(ws[0]).float()
            if ref is None:
                ref = y
            err = float((y - ref).abs().max() / ref.abs().max())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(40):
                if act == ACT_SWIGLU:
                    ops.gemm(xs, ws[i % len(ws)], act=ACT_SWIGLU)
                else:
                    C.gemm_splitk_raw(xs, ws[i % len(ws)], s, slabs, bn or 256)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(kr, []).append((e0.elapsed_time(e1) / 40 * 1e3, err))
    print(f"M=256 {name:8s} N={N:6d} K={K:6d} split {s} bn {bn}: " +
          "  ".join(f"krot{k}=" + "/".join(f"{t:.1f}us" for t, _ in v) + f"(relerr {v[-1][1]:.1e})" for k, v in res.items()),
          flush=True)
    del ws
