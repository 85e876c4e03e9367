"""Batch-1 attention + o_proj: one fused launch vs fused attention kernel + o_proj GEMV (+ residual),
over 8 distinct layers' caches and weights (cold weights like a decode step), Mistral-7B shapes.

    python tools/attn_o_bench.py [--L 330 450] [--Smax 456]
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
    ap.add_argument("--L", type=int, nargs="+", default=[330, 450])
    ap.add_argument("--Smax", type=int, default=456)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--ps", type=int, default=None, help="keys per attention partition (default heuristic)")
    a = ap.parse_args()
    dev = "cuda"
    Hq, Hkv, D, H = 32, 8, 128, 4096
    nl = a.layers
    cos, sin = ref.rope_tables(D, 4096, 10000.0, dev)
    kc = [torch.randn(1, Hkv, a.Smax, D, device=dev, dtype=torch.bfloat16) for _ in range(nl)]
    vc = [torch.randn_like(k) for k in kc]
    wo = [(torch.randn(H, Hq * D, device=dev) / 64).to(torch.bfloat16) for _ in range(nl)]
    qkv = torch.randn(1, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    res = torch.randn(1, H, device=dev, dtype=torch.bfloat16)
    ws = ops.decode_workspace(1, Hq, Hkv, D, a.Smax, dev, PS=a.ps)
    print(f"PS={ws[1]} NP={(a.Smax + ws[1] - 1) // ws[1]}")
    for L in a.L:
        slot = torch.tensor([L - 1], device=dev, dtype=torch.int32)
        attn_len = slot + 1
        pos = slot.clone()
        ks = torch.zeros(1, device=dev, dtype=torch.int32)

        def fused():
            for i in range(nl):
                ops.decode_step_attention_o(qkv, kc[i], vc[i], slot, attn_len, Hq, wo[i], res, pos, cos, sin, ks, 0,
                                            workspace=ws)

        def split():
            for i in range(nl):
                o = ops.decode_step_attention(qkv, kc[i], vc[i], slot, attn_len, Hq, pos, cos, sin, ks, 0,
                                              workspace=ws)
                ops.gemm_decode(o, wo[i], residual=res)

        def attn_only():
            for i in range(nl):
                ops.decode_step_attention(qkv, kc[i], vc[i], slot, attn_len, Hq, pos, cos, sin, ks, 0, workspace=ws)

        out = {}
        for name, fn in (("fused", fused), ("split", split), ("attn_only", attn_only)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            # a hipGraph of the 8-layer sequence (as in the decode step: launch gaps ~1 us)
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            with torch.cuda.graph(g):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) / (20 * nl) * 1e3
        print(f"L={L}: " + " ".join(f"{k}={v:6.1f}us/layer" for k, v in out.items()), flush=True)
    torch.cuda.synchronize()
    print("sync/err", ws[3].tolist())


if __name__ == "__main__" and os.environ.get("STAMPS") != "1":
    main()


def stamps():
    """Per-block phase timeline of one fused launch (s_memrealtime, 100 MHz): prints, per phase,
    min / median / max over blocks relative to the earliest block start, producers vs consumers."""
    dev = "cuda"
    Hq, Hkv, D, H, Smax, L = 32, 8, 128, 4096, 456, 450
    cos, sin = ref.rope_tables(D, 4096, 10000.0, dev)
    kc = torch.randn(1, Hkv, Smax, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    wo = (torch.randn(H, Hq * D, device=dev) / 64).to(torch.bfloat16)
    qkv = torch.randn(1, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    res = torch.randn(1, H, device=dev, dtype=torch.bfloat16)
    ps = int(os.environ["PS"]) if os.environ.get("PS") else None
    ws = ops.decode_workspace(1, Hq, Hkv, D, Smax, dev, PS=ps)
    slot = torch.tensor([L - 1], device=dev, dtype=torch.int32)
    st = torch.zeros(H // 16, 8, dtype=torch.int64, device=dev)
    C = ops.native()
    for _ in range(3):
        ops.decode_step_attention_o(qkv, kc, vc, slot, slot + 1, Hq, wo, res, slot.clone(), cos, sin,
                                    torch.zeros(1, device=dev, dtype=torch.int32), 0, workspace=ws)
    torch.cuda.synchronize()
    ops.decode_step_attention_o(qkv, kc, vc, slot, slot + 1, Hq, wo, res, slot.clone(), cos, sin,
                                torch.zeros(1, device=dev, dtype=torch.int32), 0, workspace=ws, stamps=st)
    torch.cuda.synchronize()
    t = st.cpu().double()
    t0 = t[:, 0].min()
    P = Hkv * ((Smax + ws[1] - 1) // ws[1])
    names = ["start", "published", "spin_done", "merged", "dma_done", "end"]
    for k, n in enumerate(names):
        for role, sl in (("prod", slice(0, P)), ("cons", slice(P, None))):
            col = t[sl, k]
            col = col[col > 0]
            if len(col):
                us = (col - t0) / 100.0  # 100 MHz -> us
                print(f"{n:10s} {role}: min {us.min():6.2f} med {us.median():6.2f} max {us.max():6.2f} us")


if __name__ == "__main__" and os.environ.get("STAMPS") == "1":
    stamps()
