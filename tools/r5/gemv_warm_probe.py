"""Batch-1 decode GEMVs from cold weights (rotation of copies > the 256 MB Infinity Cache) vs warm
weights (one copy, replayed back to back: resident in the Infinity Cache when it fits). Decides
whether prefetching the next projection's weights into the Infinity Cache while the HBM-idle decode
attention runs can pay. Mistral-7B shapes.

    python tools/r5/gemv_warm_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from gemv_balance_probe import t_us  # noqa: E402


def main():
    dev = "cuda"
    C = ops.native()
    x1 = torch.randn(1, 4096, device=dev, dtype=torch.bfloat16)
    x2 = torch.randn(1, 14336, device=dev, dtype=torch.bfloat16)
    shapes = (("qkv", 6144, x1, 0, 1e-5), ("o", 4096, x1, 0, 0.0), ("gate_up", 28672, x1, 5, 1e-5),
              ("down", 4096, x2, 0, 0.0))
    for name, N, x, act, eps in shapes:
        K = x.shape[1]
        ncopy = max(4, (1 << 30) // (N * K * 2))
        imgs = []
        for _ in range(ncopy):
            w = (torch.randn(N, K, device=dev) / 64).to(torch.bfloat16)
            buf = torch.empty_like(w)
            C.shuffle_decode_weight(w, buf)
            imgs.append(buf)
            del w
        fns = [lambda b=b: C.gemm(x, b, None, None, None, act, False, None, None, eps, True) for b in imgs]
        cold = t_us(fns)
        warm = t_us([fns[0]] * len(fns))
        mb = N * K * 2 / 1e6
        print(f"{name}: {mb:.1f} MB cold {cold:.2f} us ({mb / cold:.2f} TB/s) warm {warm:.2f} us ({mb / warm:.2f} TB/s)",
              flush=True)
        del imgs, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
