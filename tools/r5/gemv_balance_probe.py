"""Batch-1 decode GEMVs (gemv16_kernel on tile-ordered images): is the time set by workgroups per CU?
Times the no-split GEMV at N / 16 (or N / 32 for the SwiGLU pair) = 256 ... 1024 workgroups on a
256-CU chip, K = 4096, from cold weights (a rotation of copies larger than the 256 MB Infinity
Cache), graph-replayed. If 384 workgroups (qkv, 1.5 per CU) take as long as 512, the CUs with two
workgroups set the time.

    python tools/r5/gemv_balance_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t_us(fns, reps=5):
    """fns: list of callables, each one GEMV on a different weight copy; time per call."""
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for f in fns:
                f()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (len(fns) * reps) * 1e3


def main():
    dev = "cuda"
    C = ops.native()
    K = 4096
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    for act, Ns in ((0, (4096, 6144, 8192, 10240, 12288, 16384)), (5, (16384, 24576, 28672, 32768))):
        row = []
        for N in Ns:
            ncopy = max(4, (1 << 30) // (N * K * 2))
            imgs = []
            for _ in range(ncopy):
                w = (torch.randn(N, K, device=dev) / 64).to(torch.bfloat16)
                buf = torch.empty_like(w)
                C.shuffle_decode_weight(w, buf)
                imgs.append(buf)
                del w
            fns = [lambda b=b: C.gemm(x, b, None, None, None, act, False, None, None, 1e-5, True) for b in imgs]
            us = t_us(fns)
            wgs = N // 32 if act == 5 else N // 16
            row.append(f"N={N} ({wgs} WG) {us:.2f} us {N * K * 2 / us / 1e6:.2f} TB/s")
            del imgs, fns
            torch.cuda.empty_cache()
        print(("swiglu pair: " if act == 5 else "plain: ") + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
