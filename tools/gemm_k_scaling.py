"""Per-tile fixed cost of the 256x256 GEMM: time NT at K and 2K (same M, N, full waves).
t(2K) - 2 t(K) < 0 by the prologue + epilogue cost per tile wave.
    python tools/gemm_k_scaling.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for M, N in ((8192, 8192), (4096, 16384)):
    res = {}
    for K in (1024, 2048, 4096, 8192):
        x = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") - 0.5) / 64).to(torch.bfloat16)
        us = min(t(lambda: ops.gemm_big(x, w, 0, 0, bn=256)) for _ in range(3))
        res[K] = us
        print(f"M={M} N={N} K={K}: {us:8.1f} us  {2 * M * N * K / us / 1e9:6.0f} TF/s", flush=True)
    ks = sorted(res)
    for a, b in zip(ks, ks[1:]):
        print(f"  per-tile-wave fixed cost estimate K={a}->{b}: {(2 * res[a] - res[b]) / (M * N / 65536 / 256):.1f} us")
