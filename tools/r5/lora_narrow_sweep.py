"""LoRA narrow products at the PPO update shape (9632 tokens, Mistral-7B, rank 16 x adapters padded
to 64): split factor sweep per product, cold operands (rotation of copies), graph-replayed. Each
time includes what the product pays around it (zero fill of the fp32 accumulator, bf16 rounding).

    python tools/r5/lora_narrow_sweep.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import KMAJ, ROW, _narrow, gemm_tn  # noqa: E402
from gemv_balance_probe import t_us  # noqa: E402


def copies(shape, n, dev):
    return [torch.randn(*shape, device=dev, dtype=torch.bfloat16) for _ in range(n)]


def main():
    dev = "cuda"
    T, R = 9632, 64
    # U = X A_pad^T (forward), K = 4096 and 14336
    for K in (4096, 14336):
        xs = copies((T, K), 4, dev)
        a = torch.randn(R, K, device=dev, dtype=torch.bfloat16)
        row = []
        for ns in (1, 2, 3, 4, 6, 8):
            us = t_us([lambda x=x, ns=ns: _narrow(x, a, ROW, nsplit=ns) for x in xs])
            row.append(f"s{ns} {us:.1f}")
        print(f"U K={K} ({T * K * 2 / 1e6:.0f} MB): " + "  ".join(row), flush=True)
        del xs
    # dU = dY UB (KMAJ [N, R]), N = 6144 / 4096 / 28672
    for N in (6144, 4096, 28672):
        dys = copies((T, N), 3 if N > 8192 else 4, dev)
        ub = torch.randn(N, R, device=dev, dtype=torch.bfloat16)
        row = []
        for ns in (0, 2, 4, 8, 16, 32):
            us = t_us([lambda y=y, ns=ns: _narrow(y, ub, KMAJ, nsplit=ns) for y in dys])
            row.append(f"{'auto' if ns == 0 else 's%d' % ns} {us:.1f}")
        print(f"dU N={N} ({T * N * 2 / 1e6:.0f} MB): " + "  ".join(row), flush=True)
        del dys
    # dA = dU^T X [R, K];  dB = dY^T U [N, R]
    du = torch.randn(T, R, device=dev, dtype=torch.bfloat16)
    for K in (4096, 14336):
        xs = copies((T, K), 4, dev)
        row = []
        for ns in (0, 4, 8, 16, 24, 37):
            out = torch.zeros(R, K, device=dev)
            us = t_us([lambda x=x, ns=ns, out=out: gemm_tn(du, x, nsplit=ns, out=out) for x in xs])
            row.append(f"{'auto' if ns == 0 else 's%d' % ns} {us:.1f}")
        print(f"dA K={K}: " + "  ".join(row), flush=True)
        del xs
    for N in (6144, 4096, 28672):
        dys = copies((T, N), 3 if N > 8192 else 4, dev)
        row = []
        for ns in (0, 2, 4, 8, 16):
            out = torch.zeros(N, R, device=dev)
            us = t_us([lambda y=y, ns=ns, out=out: gemm_tn(y, du, nsplit=ns, out=out) for y in dys])
            row.append(f"{'auto' if ns == 0 else 's%d' % ns} {us:.1f}")
        print(f"dB N={N}: " + "  ".join(row), flush=True)
        del dys


if __name__ == "__main__":
    main()
