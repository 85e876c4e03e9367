"""Batch-N fused decode attention (RoPE + cache append + attention) on its own, no graph: time per
call and K/V bytes streamed per second. Used for rocprofv3 PMC runs (the graph-captured decode
loop under --pmc crashed the profiler tool on the box).

    python tools/decode_attn_probe.py [--B 256] [--ctx 237] [--iters 50]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops import reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=237)
    ap.add_argument("--Smax", type=int, default=448)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev, Hq, Hkv, D = "cuda", 32, 8, 128
    kc = torch.randn(a.B, Hkv, a.Smax, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    slot = torch.full((a.B,), a.ctx - 1, device=dev, dtype=torch.int32)
    attn_len = slot + 1
    pos = slot.clone()
    cos, sin = ref.rope_tables(D, 4096, 10000.0, dev)
    qkv = torch.randn(a.B, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    ws = ops.decode_workspace(a.B, Hq, Hkv, D, a.Smax, dev)
    out = torch.empty(a.B, Hq * D, device=dev, dtype=torch.bfloat16)
    f = lambda: ops.decode_step_attention(qkv, kc, vc, slot, attn_len, Hq, pos, cos, sin, None, 0,  # noqa: E731
                                          1 / math.sqrt(D), workspace=ws, out=out)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        f()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    gb = a.B * Hkv * a.ctx * D * 2 * 2 / 1e9
    print(f"B={a.B} ctx={a.ctx}: {us:.1f} us/call, K/V {gb * 1e3:.0f} MB -> {gb / us * 1e3:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
