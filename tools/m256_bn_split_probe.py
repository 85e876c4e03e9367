"""Batch-256 decode split-K GEMMs (raw fp32 slabs, the form the decode layer runs with the reduce
folded into the consumer): 256x128 vs 256x256 tiles over a split sweep, plus the slab bytes the
consumer must read back. Interleaved rounds, random operands, weights cold (a 1 GiB scrub between
calls evicts L2 / MALL, as in a decode step where every weight is touched once).

    python tools/m256_bn_split_probe.py [--M 256] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--model", default="mistral")
    a = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    if a.model == "mistral":
        shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}
    else:
        shapes = {"qkv": (15360, 5120), "o": (5120, 5120), "down": (5120, 13824)}
    scrub = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    M = a.M
    for name, (N, K) in shapes.items():
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) / 64).to(torch.bfloat16) for _ in range(4)]
        slabs = torch.empty(16 * M * N, dtype=torch.float32, device=dev)
        ref = x.float() @ ws[0].float().t()
        cases = {}
        for bn in (128, 256):
            tiles = N // bn
            for s in (2, 4, 5, 6, 8, 10, 12, 16):
                if tiles * s > 640 or tiles * s < 96:
                    continue
                cases[(bn, s)] = s
        res = {k: [] for k in cases}
        for _ in range(a.rounds):
            for (bn, s) in cases:
                ts = []
                for it in range(8):
                    w = ws[it % 4]
                    scrub.add_(1.0)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    C.gemm_splitk_raw(x, w, s, slabs, bn)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                res[(bn, s)].append(statistics.median(ts))
                if len(res[(bn, s)]) == 1:
                    C.gemm_splitk_raw(x, ws[0], s, slabs, bn)
                    got = slabs[:s * M * N].view(s, M, N).sum(0)
                    err = float((got - ref).abs().max() / ref.abs().max())
                    assert err < 1e-2, (name, bn, s, err)
        line = " ".join(f"bn{bn}/s{s}={statistics.median(v):6.1f}us(+{s * M * N * 4 / 1e6:4.0f}MB)"
                        for (bn, s), v in res.items())
        print(f"M={M} {name:5s} N={N} K={K} w={N * K * 2 / 1e6:.0f}MB: {line}", flush=True)


if __name__ == "__main__":
    main()
