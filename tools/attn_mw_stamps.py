"""Phase stamps (s_memrealtime, 100 MHz) of the batch-1 8-wave decode attention kernel: entry ->
prologue landed -> tiles consumed -> merged/stored, per wave, plus hipEvent time per launch."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops import reference as ref  # noqa: E402

DEV = "cuda"
B, Hq, Hkv, D, Smax = 1, 32, 8, 128, 456
C = ops.native()
kc = torch.randn(B, Hkv, Smax, D, device=DEV, dtype=torch.bfloat16)
vc = torch.randn_like(kc)
cos, sin = ref.rope_tables(D, 4096, 10000.0, DEV)
ws = ops.decode_workspace(B, Hq, Hkv, D, Smax, DEV)
qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
junk = torch.empty(512 * 2 ** 20, dtype=torch.uint8, device=DEV)
for L, cold in ((300, True), (300, False)):
    slot = torch.tensor([L - 1], device=DEV, dtype=torch.int32)
    alen = slot + 1
    pos = slot.clone()
    st = torch.zeros(Hkv * 8 * 8, dtype=torch.int64, device=DEV)
    rows = []
    ev = []
    for it in range(30):
        if cold:
            junk.fill_(it)  # evict the K/V cache from the Infinity Cache (a decode step streams GBs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.decode_step_attention(qkv, kc, vc, slot, alen, Hq, pos, cos, sin, None, 0, workspace=ws, stamps=st)
        e1.record()
        torch.cuda.synchronize()
        s = st.view(Hkv * 8, 8)[:, :4].double().cpu()
        t0 = s[:, 0].min()
        rows.append(((s - t0) / 100.0))  # us
        ev.append(e0.elapsed_time(e1) * 1e3)
    r = torch.stack(rows[5:])  # [iters, waves, 4]
    med = r.median(0).values
    print(f"L={L} {'cold' if cold else 'warm'}: event {sorted(ev[5:])[len(ev[5:]) // 2]:.2f} us/launch; stamps (us from first wave entry), "
          f"median over iterations:")
    for k, name in enumerate(["entry", "prologue", "tiles", "merged"]):
        col = med[:, k]
        print(f"   {name:9s} min {col.min():6.2f}  med {col.median():6.2f}  max {col.max():6.2f}")
