"""PPO-update GEMM shapes (Mistral-7B, minibatch 16 x ~300 tokens) on every available path, in one
process, interleaved rounds (guide §5.4 rule 24), random operands.

Forward (NT: y = x W^T, LoRA rank 64 as extra K): ours 128-tile / ours 256-tile / hipBLASLt.
Backward dX (NN: dx = dy W): hipBLASLt, and ours via an explicit transposed weight copy (W^T
materialised once, as a resident transposed weight would be).

    python tools/update_gemm_probe.py [--M 4800] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


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
    ap.add_argument("--M", type=int, nargs="+", default=[4800, 7168])
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    H, F, NQKV = 4096, 14336, 6144
    shapes = [("qkv", NQKV, H), ("o", H, H), ("gate_up", 2 * F, H), ("down", H, F)]
    for M in a.M:
        for name, N, K in shapes:
            x = torch.rand(M, K, device=dev, dtype=torch.bfloat16) * 2 - 1
            w = (torch.rand(N, K, device=dev, dtype=torch.bfloat16) * 2 - 1) / 64
            u = torch.rand(M, 64, device=dev, dtype=torch.bfloat16) * 2 - 1
            ub = (torch.rand(N, 64, device=dev, dtype=torch.bfloat16) * 2 - 1) / 64
            dy = torch.rand(M, N, device=dev, dtype=torch.bfloat16) * 2 - 1
            wt = w.t().contiguous()  # [K, N]
            cases = {
                "fwd_lora_t128": lambda: (C.set_tuning({"gemm_variant": 1}), C.gemm(x, w, u, ub, None, 0, False, None)),
                "fwd_lora_t256": lambda: (C.set_tuning({"gemm_variant": 2}), C.gemm(x, w, u, ub, None, 0, False, None)),
                "fwd_lib_plain": lambda: torch.matmul(x, w.t()),
                "dx_lib_nn": lambda: torch.matmul(dy, w),
                "dx_ours_t256_wT": lambda: (C.set_tuning({"gemm_variant": 2}), C.gemm(dy, wt, None, None, None, 0, False, None)),
                "dx_lib_nt_wT": lambda: torch.matmul(dy, wt.t()),
            }
            res = {k: [] for k in cases}
            for _ in range(a.rounds):
                for k, fn in cases.items():
                    res[k].append(timeit(fn))
            C.set_tuning({"gemm_variant": 0})
            fl = 2 * M * N * K
            line = " ".join(f"{k}={statistics.median(v):7.1f}us({fl / statistics.median(v) / 1e6:5.0f}TF)"
                            for k, v in res.items())
            print(f"M={M} {name:8s} N={N} K={K}: {line}", flush=True)


if __name__ == "__main__":
    main()
