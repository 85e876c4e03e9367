"""Batch-256 decode: o / down projection split-K factor judged with its consumer. The split-K
slabs (nsplit x 256 x 4096 fp32) are written by the GEMM and read by the slab-summing RMSNorm, so
the plan's split (8, chosen on the GEMM alone) also sets the norm's bytes. Times GEMM + norm per
split over a rotation of weight copies (cold weights), graph-replayed. Mistral-7B shapes.

    python tools/r5/m256_split_norm_probe.py
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
    lnw = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    res = torch.randn(M, 4096, device=dev, dtype=torch.bfloat16)
    for name, N, K in (("o", 4096, 4096), ("down", 4096, 14336)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        ncopy = max(4, (1 << 29) // (N * K * 2))
        ws = [(torch.randn(N, K, device=dev) / 64).to(torch.bfloat16) for _ in range(ncopy)]
        row = []
        for s in tuple(int(v) for v in os.environ.get("SPLITS", "2,3,4,5,6,8,10,12").split(",")):
            slabs = torch.empty(s * M * N, device=dev)

            def gemm_only(w, s=s, slabs=slabs):
                C.gemm_splitk_raw(x, w, s, slabs, 128)

            def both(w, s=s, slabs=slabs):
                C.gemm_splitk_raw(x, w, s, slabs, 128)
                ops.rms_norm(SplitK(slabs, s, M, N, torch.bfloat16), lnw, 1e-5, res)

            tg = t_us([lambda w=w: gemm_only(w) for w in ws])
            tb = t_us([lambda w=w: both(w) for w in ws])
            row.append(f"s{s} {tg:.1f}+{tb - tg:.1f}={tb:.1f}")
        print(f"{name}: " + "  ".join(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
