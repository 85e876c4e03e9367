"""Run one GEMM configuration a few times (for rocprofv3 --pmc counter collection).

Usage: python tools/prof_gemm.py --M 7168 --N 28672 --K 4096 --rp 64 --variant 2 --iters 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=7168)
    ap.add_argument("--N", type=int, default=28672)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--rp", type=int, default=64)
    ap.add_argument("--variant", type=int, default=2)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    C = ops.native()
    C.set_tuning({"gemm_variant": a.variant})
    x = torch.randn(a.M, a.K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.N, a.K, device="cuda", dtype=torch.bfloat16) / 64
    u = torch.randn(a.M, a.rp, device="cuda", dtype=torch.bfloat16) if a.rp else None
    ub = torch.randn(a.N, a.rp, device="cuda", dtype=torch.bfloat16) if a.rp else None
    for _ in range(a.iters):
        C.gemm(x, w, u, ub, None, 0, False, None)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
