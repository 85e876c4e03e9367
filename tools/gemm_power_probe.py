"""Is the big GEMM clock/power bound? The same NT GEMM (M = 9632, Mistral-7B shapes) on
zero-filled, constant, and uniform-random operands: matrix-core time does not depend on the data,
so a gap between them is the clock the chip can hold under that switching activity.
    python tools/gemm_power_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    M = 9632
    for name, N, K in (("qkv", 6144, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
        res = []
        for kind in ("zero", "const", "rand", "zero", "rand"):
            if kind == "zero":
                x = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
                w = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
            elif kind == "const":
                x = torch.full((M, K), 0.5, device="cuda", dtype=torch.bfloat16)
                w = torch.full((N, K), 0.25, device="cuda", dtype=torch.bfloat16)
            else:
                x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
                w = ((torch.rand(N, K, device="cuda") * 2 - 1) / 64).to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            us = t(lambda: ops.gemm(x, w, out=out))
            res.append(f"{kind}={us:7.1f}us({2 * M * N * K / us / 1e6:5.0f}TF)")
            del x, w, out
        print(f"{name:8s} " + " ".join(res), flush=True)


if __name__ == "__main__":
    main()
