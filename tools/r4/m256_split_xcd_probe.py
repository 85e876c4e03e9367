"""Batch-256 decode split-K GEMMs (256x128 tiles, raw fp32 slabs): XCD order of the (split, tile)
blocks, tuning gemm_split_xcd 0 (tile-major: every XCD runs every split and reads all of A) vs 1
(split-major: the blocks sharing an A K-slice share an L2). Interleaved rounds, weights cold (a
1 GiB scrub between launches), results checked against fp32. The switch (a split-major
xcd_remap over nwg x nsplit in gemm_big_kernel) was removed after this measurement
(profiles/r4/m256_split_xcd_order.log: neutral); the script records how it was measured.

    python tools/r4/m256_split_xcd_probe.py [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import splitk_plan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--M", type=int, default=256)
    a = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    shapes = {"qkv": (6144, 4096, (4, 5, 6, 8)), "o": (4096, 4096, (6, 8, 10, 16)),
              "down": (4096, 14336, (6, 8, 12, 16))}
    scrub = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    M = a.M
    for name, (N, K, splits) in shapes.items():
        plan = splitk_plan(M, N, K)[0]
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        ws = [((torch.rand(N, K, device=dev) * 2 - 1) / 64).to(torch.bfloat16) for _ in range(4)]
        slabs = torch.empty(16 * M * N, dtype=torch.float32, device=dev)
        ref = x.float() @ ws[0].float().t()
        res = {(s, v): [] for s in splits for v in (0, 1)}
        for _ in range(a.rounds):
            for (s, v) in res:
                with ops.tuning(gemm_split_xcd=v):
                    ts = []
                    for it in range(8):
                        w = ws[it % 4]
                        scrub.add_(1.0)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        C.gemm_splitk_raw(x, w, s, slabs, 128)
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    res[(s, v)].append(statistics.median(ts))
                    if len(res[(s, v)]) == 1:
                        C.gemm_splitk_raw(x, ws[0], s, slabs, 128)
                        got = slabs[:s * M * N].view(s, M, N).sum(0)
                        err = float((got - ref).abs().max() / ref.abs().max())
                        assert err < 1e-2, (name, s, v, err)
        line = "  ".join(f"s{s}{'*' if s == plan else ''}: {statistics.median(res[(s, 0)]):5.1f} -> "
                         f"{statistics.median(res[(s, 1)]):5.1f}us" for s in splits)
        print(f"M={M} {name:5s} N={N} K={K} w={N * K * 2 / 1e6:.0f}MB  tile-major -> split-major  {line}", flush=True)


if __name__ == "__main__":
    main()
