"""LoRA narrow products on the 64x64-tile kernel at PPO-update token counts: U = X A_pad^T and
dU = dY UB (ops.linear._narrow) with and without the split reduction, and the dA / dB token
reductions (ops.gemm_tn). Bandwidth = bytes of the wide operand / time.

    python tools/lora_narrow_probe.py [--M 9632]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import _narrow  # noqa: E402


def timeit(fn, iters=10):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=9632)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev, M, R = "cuda", a.M, 64
    for K in (4096, 6144, 14336, 28672):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ap_ = (torch.randn(R, K, device=dev) / 64).to(torch.bfloat16)  # ROW [R, K]
        ub = (torch.randn(K, R, device=dev) / 64).to(torch.bfloat16)   # KMAJ [K, R] (UB of an N=K layer)
        du = torch.randn(M, R, device=dev).to(torch.bfloat16)
        cases = {"u_ns1": lambda: _narrow(x, ap_, ops.ROW, 1), "u_auto": lambda: _narrow(x, ap_, ops.ROW),
                 "du_ns1": lambda: _narrow(x, ub, ops.KMAJ, 1), "du_auto": lambda: _narrow(x, ub, ops.KMAJ),
                 "dA_tn": lambda: ops.gemm_tn(du, x), "dB_tn": lambda: ops.gemm_tn(x, du)}
        res = {k: [] for k in cases}
        for _ in range(a.rounds):
            for k, fn in cases.items():
                res[k].append(timeit(fn))
        gb = M * K * 2 / 1e9
        print(f"M={M} K={K}: " + " ".join(f"{k}={statistics.median(v):7.1f}us({gb / statistics.median(v) * 1e6 / 1e3:4.2f}TB/s)"
                                         for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
