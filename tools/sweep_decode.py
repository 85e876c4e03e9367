"""Decode-GEMM sweep under hipGraph replay (no host launch overhead in the numbers).

For each Mistral-7B decode shape, captures `reps` back-to-back GEMMs over distinct weight copies
(> 256 MB total, so every launch streams its weights from HBM like a real decode step) and reports
kernel time per GEMM and effective weight bandwidth, for each split-K / pipeline-depth setting and
for the tile-ordered (shuffled) weight image.

    python tools/sweep_decode.py [--M 1] [--splits 0,2,4,8,16]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
          ("lm_head", 32000, 4096)]


def graph_time(fn, replays=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / replays * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="1")
    ap.add_argument("--splits", default="0,1,2,4,8,16")
    ap.add_argument("--only", default=None)
    ap.add_argument("--depths", default="0", help="weight-pipeline depths of the M<=16 kernel (0 = auto)")
    ap.add_argument("--shuf-splits", default="0", help="split-K settings for the shuffled-weight runs")
    args = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    pass  # single (hand-written) GEMM path since round 2
    for M in [int(m) for m in args.M.split(",")]:
        for name, N, K in SHAPES:
            if args.only and name not in args.only.split(","):
                continue
            reps = max(4, int(1.2e9 // (N * K * 2)))
            ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(reps)]
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            outs = [torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(reps)]
            byts = N * K * 2
            for sp, dp in [(int(v), int(d)) for v in args.splits.split(",") for d in args.depths.split(",")]:
                C.set_tuning({"m64_split" if M > 16 else "decode_split": sp})
                C.set_tuning({"decode_depth": dp})

                def run():
                    for w, o in zip(ws, outs):
                        ops.gemm(x, w, out=o)
                t = graph_time(run) / reps
                r = dict(kind="decode_gemm", name=name, M=M, N=N, K=K, split=sp, depth=dp, us=round(t, 2),
                         tbs=round(byts / t / 1e6, 2))
                print(json.dumps(r), flush=True)
            C.set_tuning({"decode_split": 0})
            C.set_tuning({"decode_depth": 0})
            C.set_tuning({"m64_split": 0})
            # tile-ordered weight image (shuffle_decode_weight): same kernel, contiguous 1-KiB loads
            ref = C.gemm(x, ws[0])
            ws = [C.shuffle_decode_weight(w) for w in ws]

            def run_shuf():
                for w, o in zip(ws, outs):
                    C.gemm(x, w, out=o, w_shuffled=True)
            for sp in [int(v) for v in args.shuf_splits.split(",")]:
                C.set_tuning({"decode_split": sp})
                t = graph_time(run_shuf) / reps
                err = float((ref.float() - outs[0].float()).abs().max() / ref.float().abs().max())
                print(json.dumps(dict(kind="decode_gemm", name=name, M=M, N=N, K=K, split=f"shuf{sp}",
                                      us=round(t, 2), tbs=round(byts / t / 1e6, 2), rel_err=err)), flush=True)
            C.set_tuning({"decode_split": 0})
            del ws, outs
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
