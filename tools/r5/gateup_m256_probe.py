"""Batch-256 decode gate / up + SwiGLU: the 256x128 no-split kernel (SwiGLU in the epilogue) vs
split-K into fp32 slabs + the SwiGLU reduce kernel, over (nsplit, bn). GPU time per call from a
captured graph of 20 calls. Mistral-7B (F = 14336, K = 4096) and Llama-2-13B (F = 13824, K = 5120).

    python tools/r5/gateup_m256_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t_us(fn, n=20, reps=10):
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
    C = ops.native()
    for (F, K) in ((14336, 4096), (13824, 5120)):
        M = 256
        w = (torch.randn(2 * F, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        ref = ops.gemm(x, w, None, None, None, 5)
        res = [f"F={F} K={K}: no-split bn128 {t_us(lambda: ops.gemm(x, w, None, None, None, 5)):.1f} us"]
        for ns, bn in ((2, 256), (2, 128), (3, 256), (4, 256)):
            slabs = torch.empty(ns * M * 2 * F, device=dev)
            out = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
            us = t_us(lambda: C.gemm_splitk(x, w, ns, slabs, None, 5, out, None, bn))
            err = (out.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
            res.append(f"s{ns}/bn{bn} {us:.1f} us (rel err {err:.1e})")
        print("  ".join(res), flush=True)


if __name__ == "__main__":
    main()
