"""Attention backward at the PPO update shape: dQ kernel head-packed (16 positions x 4 heads) vs 64
positions of one head; whole backward (delta + dK / dV + dQ) timed, graph-replayed.

    python tools/r5/attn_dq_hp_probe.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from gemv_balance_probe import t_us  # noqa: E402


def main():
    dev = "cuda"
    C = ops.native()
    Hq, Hkv, D = 32, 8, 128
    for B, S in ((32, 301), (64, 150)):
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
        o, lse = C.attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, True, 0, 1 / math.sqrt(D), None, None, None, 0, True)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        res = []
        for maxs in (4096, 0):
            with ops.tuning(attn_dq_hp_maxs=maxs):
                us = t_us([lambda: C.attn_bwd(q, k, v, o, do, lse, dqkv[:, :Hq * D], dqkv[:, Hq * D:(Hq + Hkv) * D],
                                               dqkv[:, (Hq + Hkv) * D:], B, S, Hq, Hkv, D, True, 0, 1 / math.sqrt(D))])
            res.append(f"{'hp' if maxs else '64row'} {us:.1f} us")
        print(f"bwd B={B} S={S}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
