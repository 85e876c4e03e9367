"""Batch-1 decode GEMVs from cold weights under the gemv16 knobs: waves per 16-row group (4 / 8 /
16) and weight-pipeline depth (4 / 6 / 8 at 4 waves). Mistral-7B shapes, graph-replayed rotation of
weight copies larger than the Infinity Cache.

    python tools/r5/gemv_knob_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from gemv_balance_probe import t_us  # noqa: E402

KNOBS = [dict(gemv16_waves=0, gemv16_depth=4), dict(gemv16_waves=4, gemv16_depth=4), dict(gemv16_waves=8, gemv16_depth=4),
         dict(gemv16_waves=16, gemv16_depth=4), dict(gemv16_waves=4, gemv16_depth=6), dict(gemv16_waves=4, gemv16_depth=8)]


def main():
    dev = "cuda"
    C = ops.native()
    x1 = torch.randn(1, 4096, device=dev, dtype=torch.bfloat16)
    x2 = torch.randn(1, 14336, device=dev, dtype=torch.bfloat16)
    shapes = (("qkv", 6144, x1, 0, 1e-5), ("o", 4096, x1, 0, 0.0), ("down", 4096, x2, 0, 0.0), ("lm_head", 32000, x1, 0, 0.0))
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
        res = []
        for kn in KNOBS:
            with ops.tuning(**kn):
                fns = [lambda b=b: C.gemm(x, b, None, None, None, act, False, None, None, eps, True) for b in imgs]
                us = t_us(fns)
            res.append(f"w{kn['gemv16_waves']}/d{kn['gemv16_depth']} {us:.2f}")
        print(f"{name} ({N * K * 2 / 1e6:.1f} MB): " + "  ".join(res), flush=True)
        del imgs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
