"""LoRA forward variants on the PPO-update shapes (M = 4800 / 7168), hipBLASLt, random operands:
plain X W^T (no adapter, the floor) | ext [X | U] @ [W | UB]^T (K + 64) | plain + rank-64 addmm
(y += U UB^T, beta = 1) | ext padded so K + Rp is a multiple of 256.

    python tools/lora_fwd_probe.py [--M 4800 7168] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.splitk_probe import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[4800, 7168])
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda"
    H, F, NQKV = 4096, 14336, 6144
    for M in a.M:
        for name, N, K in [("qkv", NQKV, H), ("o", H, H), ("gate_up", 2 * F, H), ("down", H, F)]:
            r = lambda *s: (torch.rand(*s, device=dev, dtype=torch.bfloat16) * 2 - 1)
            x, w, u, ub = r(M, K), r(N, K) / 64, r(M, 64), r(N, 64) / 64
            xe, we = torch.cat([x, u], 1), torch.cat([w, ub], 1)
            pad = (256 - (K + 64) % 256) % 256
            xp = torch.cat([x, u, torch.zeros(M, pad, device=dev, dtype=x.dtype)], 1)
            wp = torch.cat([w, ub, torch.zeros(N, pad, device=dev, dtype=x.dtype)], 1)

            def plain_addmm():
                y = x @ w.t()
                return y.addmm_(u, ub.t())

            cases = {"plain": lambda: x @ w.t(), "ext": lambda: xe @ we.t(), "plain+addmm": plain_addmm,
                     f"ext_pad{pad}": lambda: xp @ wp.t()}
            res = {k: [] for k in cases}
            for _ in range(a.rounds):
                for k, fn in cases.items():
                    res[k].append(timeit(fn))
            print(f"M={M} {name:8s} N={N} K={K}: " + " ".join(f"{k}={statistics.median(v):7.1f}us"
                                                              for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
