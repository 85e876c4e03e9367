"""Batch-1 sampler timing (sample_topk_search_kernel): window path vs full-row search, over logit
scales, top-p on / off. Events around 200 back-to-back calls.

    python tools/r5/sampler_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t_us(fn, n=50, reps=10):
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
    dev = "cuda"
    V = 32000
    off = torch.zeros(1, dtype=torch.long, device=dev)
    for B in (1, 256):
        for scale in (0.3, 1.3, 3.0, 8.0):
            g = torch.Generator(device="cpu").manual_seed(1)
            logits = (torch.randn(B, V, generator=g) * scale).to(torch.bfloat16).to(dev)
            row = []
            for w in (1, 0):
                for tp in (1.0, 0.9):
                    with ops.tuning(sample_window=w):
                        us = t_us(lambda: ops.sample(logits, 1 / 0.7, top_k=50, top_p=tp, seed=3, offset=off))
                    row.append(f"win={w} top_p={tp}: {us:6.1f} us")
            print(f"B={B:3d} scale={scale:4.1f}  " + "  ".join(row), flush=True)
    # greedy (argmax) path for reference
    logits = (torch.randn(1, V) * 1.3).to(torch.bfloat16).to(dev)
    print(f"greedy B=1: {t_us(lambda: ops.sample(logits, 1.0, top_k=0, top_p=1.0, seed=3, offset=off, greedy=True)):.1f} us")


if __name__ == "__main__":
    main()
