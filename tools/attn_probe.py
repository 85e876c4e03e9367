"""Flash attention fwd + bwd at the PPO-update shape (16 x 448 tokens, Mistral-7B heads), for
kernel timing / PMC counter runs:  python tools/attn_probe.py [--iters 5] [--B 16] [--S 448]"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, default=448)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd import ops
    B, S, Hq, Hkv, D = a.B, a.S, a.Hq, a.Hkv, a.D
    qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * D, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
    ks = torch.zeros(B, dtype=torch.int32, device="cuda")
    go = torch.randn(B * S, Hq * D, device="cuda", dtype=torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for i in range(a.iters + 1):
        if i == 1:
            ev[0].record()
        o = ops.flash_attention_qkv(qkv, B, S, Hq, Hkv, D, True, 0, 1 / math.sqrt(D), kv_start=ks)
        if i == 1:
            ev[1].record()
        o.backward(go)
        qkv.grad = None
    ev[2].record()
    torch.cuda.synchronize()
    fl = 4 * B * Hq * S * S * D / 2
    tf = ev[0].elapsed_time(ev[1]) * 1e-3
    tb = (ev[0].elapsed_time(ev[2]) / a.iters) * 1e-3 - tf
    print(f"fwd {tf * 1e6:.1f} us ({fl / tf / 1e12:.0f} TF/s); bwd ~{tb * 1e6:.1f} us ({2.5 * fl / tb / 1e12:.0f} TF/s)")


if __name__ == "__main__":
    main()
