"""Causal training attention at the PPO shapes: tile-order dispatch vs heaviest-first (LPT) within
each XCD (tuning attn_lpt). Forward (head-packed GQA-4 tiles) and the whole backward (delta + dK /
dV + dQ), each graph-replayed, settings interleaved over rounds; median us per call.

    python tools/r6/attn_lpt_probe.py [--rounds 5]
"""
import argparse
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t_us(fn, n=20, reps=5):
    """GPU time per call: n calls captured in one HIP graph (no host dispatch gaps), replayed."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
        with torch.cuda.graph(g, stream=st):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (n * reps) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    dev = "cuda"
    C = ops.native()
    Hq, Hkv, D = 32, 8, 128
    sc = 1 / math.sqrt(D)
    # (label, B, S, left padding): update minibatch, reference scoring minibatch, rollout prefill
    shapes = [("update mb32", 32, 301, False), ("update mb32 left-pad", 32, 301, True), ("update mb64", 64, 301, False),
              ("reference mb128", 128, 301, False), ("prefill 256x173", 256, 173, False)]
    torch.manual_seed(0)
    for label, B, S, left in shapes:
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
        ks = torch.randint(0, 96, (B,), device=dev, dtype=torch.int32) if left else None
        o, lse = C.attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, True, 0, sc, ks, None, None, 0, True)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        fwd = lambda: C.attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, True, 0, sc, ks, None, None, 0, True)  # noqa: E731
        bwd = lambda: C.attn_bwd(q, k, v, o, do, lse, dqkv[:, :Hq * D], dqkv[:, Hq * D:(Hq + Hkv) * D],  # noqa: E731
                                 dqkv[:, (Hq + Hkv) * D:], B, S, Hq, Hkv, D, True, 0, sc, ks)
        res = {(w, l): [] for w in ("fwd", "bwd") for l in (0, 1)}
        for _ in range(args.rounds):
            for lpt in (0, 1):  # forced either way (the default gates it on the grid size)
                with ops.tuning(attn_lpt=(1 << 30) * lpt):
                    res[("fwd", lpt)].append(t_us(fwd))
                    res[("bwd", lpt)].append(t_us(bwd))
        med = {k_: statistics.median(v_) for k_, v_ in res.items()}
        print(f"{label:22s} fwd tile-order {med[('fwd', 0)]:7.1f} us  heaviest-first {med[('fwd', 1)]:7.1f} us | "
              f"bwd tile-order {med[('bwd', 0)]:7.1f} us  heaviest-first {med[('bwd', 1)]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
