"""Training / reference / prefill attention forward: head-packed 32-position tiles (GQA-4) vs the
128-position tiles of one head. Mistral-7B heads, causal, graph-replayed.

    python tools/r5/attn_fwd_hp_probe.py
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
    for name, B, S in (("update_b32_s301", 32, 301), ("ref_b128_s301", 128, 301), ("prefill_b256_s173", 256, 173),
                       ("answer_b1_s174", 1, 174), ("long_b1_s1024", 1, 1024)):
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
        ks = torch.randint(0, 20, (B,), device=dev, dtype=torch.int32)
        res = []
        for maxs in (4096, 0):
            with ops.tuning(attn_fwd_hp_maxs=maxs):
                us = t_us([lambda: C.attn_fwd(q, k, v, B, S, S, Hq, Hkv, D, True, 0, 1 / math.sqrt(D), ks, None, None, 0,
                                             True)])
            res.append(f"{'hp' if maxs else '128row'} {us:.1f} us")
        print(f"{name}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
