"""Wave quantisation of the PPO-update GEMMs with a 4096-wide output (M = 16 x ~300 tokens = 4800:
19 x 16 = 304 tiles of 256^2 on 256 CUs = 1.19 waves). Compares one hipBLASLt GEMM with a K-split
batched GEMM (fp32 partials) + reduction, in one process, interleaved rounds, random operands.

    python tools/splitk_probe.py [--M 4800 7168] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


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


def split_nn(a, b, c):
    """a [M, K] @ b [K, N] as c K-chunks -> fp32 partials -> bf16."""
    M, K = a.shape
    kc = K // c
    part = torch.bmm(a.unflatten(1, (c, kc)).transpose(0, 1), b.unflatten(0, (c, kc)), out_dtype=torch.float32)
    return part.sum(0).to(a.dtype)


def split_nt(a, w, c):
    """a [M, K] @ w[N, K]^T as c K-chunks."""
    M, K = a.shape
    kc = K // c
    part = torch.bmm(a.unflatten(1, (c, kc)).transpose(0, 1), w.unflatten(1, (c, kc)).permute(1, 2, 0),
                     out_dtype=torch.float32)
    return part.sum(0).to(a.dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[4800, 7168])
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda"
    H, F, NQKV, R = 4096, 14336, 6144, 64
    # (name, kind, N_out, K): kind nn = dY @ W (W [K, N] row-major view), nt = X @ W^T
    shapes = [("dx_gate_up", "nn", H, 2 * F), ("dx_qkv", "nn", H, NQKV), ("dx_o", "nn", H, H),
              ("fwd_down_ext", "nt", H, F + R), ("fwd_o_ext", "nt", H, H + R)]
    for M in a.M:
        for name, kind, N, K in shapes:
            x = torch.rand(M, K, device=dev, dtype=torch.bfloat16) * 2 - 1
            if kind == "nn":
                w = (torch.rand(K, N, device=dev, dtype=torch.bfloat16) * 2 - 1) / 64
                cases = {"lib": lambda: x @ w}
                for c in (2, 3, 4):
                    if K % c == 0:
                        cases[f"split{c}"] = (lambda c=c: split_nn(x, w, c))
            else:
                w = (torch.rand(N, K, device=dev, dtype=torch.bfloat16) * 2 - 1) / 64
                cases = {"lib": lambda: x @ w.t()}
                for c in (2, 3, 4):
                    if K % c == 0 and (K // c) % 8 == 0:
                        cases[f"split{c}"] = (lambda c=c: split_nt(x, w, c))
            ref = cases["lib"]().float()
            for k, fn in cases.items():
                err = (fn().float() - ref).abs().max().item()
                assert err < 0.05 * ref.abs().max().item() + 1e-3, (name, k, err)
            res = {k: [] for k in cases}
            for _ in range(a.rounds):
                for k, fn in cases.items():
                    res[k].append(timeit(fn))
            fl = 2 * M * N * K
            line = " ".join(f"{k}={statistics.median(v):7.1f}us({fl / statistics.median(v) / 1e6:5.0f}TF)"
                            for k, v in res.items())
            print(f"M={M} {name:12s} N={N} K={K}: {line}", flush=True)


if __name__ == "__main__":
    main()
