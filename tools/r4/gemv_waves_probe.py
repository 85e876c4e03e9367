"""Batch-1 decode GEMVs (gemv16_kernel over tile-ordered weights, Mistral-7B qkv / o / down; gate_up
is the SwiGLU pair form, always 4 waves) with 4 / 8 / 16 waves per 16-row group (tuning gemv16_waves).
Each launch cold (a 1 GiB read between launches evicts L2 and the Infinity Cache, as in a decode
step where every weight is read once); interleaved rounds, median microseconds.

    python tools/r4/gemv_waves_probe.py [--reps 40]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--fp8", action="store_true", help="W8A16: the tile-ordered e4m3fn image (config 5)")
    ap.add_argument("--model", default="mistral-7b", choices=["mistral-7b", "llama2-13b"])
    ap.add_argument("--M", type=int, default=1)
    a = ap.parse_args()
    flush = torch.ones(1 << 29, dtype=torch.bfloat16, device="cuda")
    shapes = (("qkv", 6144, 4096, 0), ("o", 4096, 4096, 1), ("gate_up", 28672, 4096, 0), ("down", 4096, 14336, 1),
              ("lm_head", 32000, 4096, 0))
    if a.model == "llama2-13b":
        shapes = (("qkv", 15360, 5120, 0), ("o", 5120, 5120, 1), ("gate_up", 27648, 5120, 0), ("down", 5120, 13824, 1),
                  ("lm_head", 32000, 5120, 0))
    for name, N, K, resid in shapes:
        x = torch.randn(a.M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        r = torch.randn(a.M, N, device="cuda", dtype=torch.bfloat16) if resid else None
        act = ops.ACT_SWIGLU if name == "gate_up" else 0
        sc = ops.ShufCache() if not a.fp8 else None
        f8 = ops.Fp8Cache() if a.fp8 else None
        if sc is not None:
            sc.get(w)
        res = {4: [], 8: [], 16: []}
        outs = {}
        for _ in range(a.rounds):
            for waves in (4, 8, 16):
                with ops.tuning(gemv16_waves=waves):
                    outs[waves] = ops.gemm_decode(x, w, act=act, residual=r, shuf=sc, fp8=f8)
                    ts = []
                    for _ in range(a.reps):
                        flush.sum()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        ops.gemm_decode(x, w, act=act, residual=r, shuf=sc, fp8=f8)
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1) * 1e3)
                    res[waves].append(statistics.median(ts))
        diff = max(float((outs[4].float() - outs[v].float()).abs().max()) for v in (8, 16))
        mb = N * K * (1 if a.fp8 else 2) / 1e6
        line = " | ".join(f"{v} waves {statistics.median(res[v]):6.1f} us ({mb / statistics.median(res[v]):4.2f} TB/s)"
                          for v in (4, 8, 16))
        print(f"M={a.M} {'fp8 ' if a.fp8 else ''}{name:8s} {mb:6.1f} MB: {line} | max |diff| {diff:.3g}", flush=True)


if __name__ == "__main__":
    main()
