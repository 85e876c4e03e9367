"""Training flash attention (ops.flash_attention_qkv) forward + backward at PPO-update shapes
(32 sequences x 301 tokens, 32 q-heads / 8 kv-heads, D 128): time per fwd and per fwd+bwd.
(The round-1 fp32-atomic dQ form left the product kernels in round 5; the dQ kernel is the only form.)

    python tools/attn_train_probe.py [--B 32] [--S 301]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--S", type=int, default=301)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tuning", default="", help="kernel-selection overrides, e.g. attn_fwd_w8=1")
    a = ap.parse_args()
    if a.tuning:
        ops.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in a.tuning.split(","))})
    Hq, Hkv, D = 32, 8, 128
    x = torch.randn(a.B * a.S, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
    go = torch.randn(a.B * a.S, Hq * D, device="cuda", dtype=torch.bfloat16)

    def fwd():
        with torch.no_grad():
            ops.flash_attention_qkv(x.detach(), a.B, a.S, Hq, Hkv, D, True, 0)

    def fwdbwd():
        x.grad = None
        o = ops.flash_attention_qkv(x, a.B, a.S, Hq, Hkv, D, True, 0)
        o.backward(go)

    res = {}
    for name, fn in (("fwd", fwd), ("fwd+bwd", fwdbwd)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / a.iters * 1e3
    flops = 4 * a.B * Hq * a.S * a.S / 2 * D
    print(f"B={a.B} S={a.S} tuning={a.tuning or 'default'}: fwd {res['fwd']:.1f} us "
          f"({flops / res['fwd'] / 1e6:.0f} TF/s), fwd+bwd {res['fwd+bwd']:.1f} us, bwd ~{res['fwd+bwd'] - res['fwd']:.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
