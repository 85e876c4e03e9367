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
    D = 128
    for name, B, S, Hq, Hkv in (("update_b32_s301", 32, 301, 32, 8), ("ref_b128_s301", 128, 301, 32, 8),
                                ("prefill_b256_s173", 256, 173, 32, 8), ("answer_b1_s174", 1, 174, 32, 8),
                                ("long_b1_s1024", 1, 1024, 32, 8), ("mha13b_update_b32_s301", 32, 301, 40, 40),
                                ("mha13b_prefill_b256_s173", 256, 173, 40, 40)):
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
