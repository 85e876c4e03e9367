"""Batch-256 decode split-K factors, second pass: Mistral-7B qkv (GEMM alone: its consumer is the
attention prologue) and the Llama-2-13B fp8 (W8A8) o / down with the slab-summing norm.

    python tools/r5/m256_split_probe2.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import SplitK  # noqa: E402
from gemv_balance_probe import t_us  # noqa: E402


def main():
    dev = "cuda"
    C = ops.native()
    M = 256
    # Mistral qkv, bf16
    x = torch.randn(M, 4096, device=dev, dtype=torch.bfloat16)
    ws = [(torch.randn(6144, 4096, device=dev) / 64).to(torch.bfloat16) for _ in range(8)]
    row = []
    for s in (3, 4, 5, 6, 8):
        slabs = torch.empty(s * M * 6144, device=dev)
        t = t_us([lambda w=w, s=s, slabs=slabs: C.gemm_splitk_raw(x, w, s, slabs, 128) for w in ws])
        row.append(f"s{s} {t:.1f}")
    print("qkv gemm: " + "  ".join(row), flush=True)
    del ws
    # 13B fp8 o / down + norm (H = 5120)
    lnw = torch.ones(5120, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, 5120, device=dev, dtype=torch.bfloat16)
    for name, N, K in (("13b_o_fp8", 5120, 5120), ("13b_down_fp8", 5120, 13824)):
        xb = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        xq, sx = ops.quantize_fp8(xb)
        qs = []
        for _ in range(max(4, (1 << 29) // (N * K))):
            q, sc = ops.quantize_fp8((torch.randn(N, K, device=dev) / 64).to(torch.bfloat16))
            qs.append((q, sc))
        row = []
        for s in (3, 4, 5, 6, 8, 10):
            slabs = torch.empty(s * M * N, device=dev)

            def both(q, sc, s=s, slabs=slabs):
                C.gemm_fp8_splitk_raw(xq, sx, q, sc, s, slabs, 128)
                ops.rms_norm(SplitK(slabs, s, M, N, torch.bfloat16), lnw, 1e-5, res)

            def g_only(q, sc, s=s, slabs=slabs):
                C.gemm_fp8_splitk_raw(xq, sx, q, sc, s, slabs, 128)

            tg = t_us([lambda q=q, sc=sc: g_only(q, sc) for q, sc in qs])
            tb = t_us([lambda q=q, sc=sc: both(q, sc) for q, sc in qs])
            row.append(f"s{s} {tg:.1f}+{tb - tg:.1f}={tb:.1f}")
        print(f"{name}: " + "  ".join(row), flush=True)
        del qs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
