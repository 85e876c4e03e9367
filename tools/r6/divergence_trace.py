#!/usr/bin/env python3
"""Per-layer hidden-state divergence: decode engine vs training forward vs fp32 oracle.

VERDICT r5 item 5: the rollout's sampler log-probs differ from the training forward's by ~0.09
nats / token on a random-init Mistral-7B. This traces WHERE the two bf16 engines drift apart, on a
4-layer model of Mistral-7B width (H 4096, 32 q / 8 kv heads x 128, FFN 14336, vocab 32000,
random init std 0.02, optional LoRA r=16 with random B so the merged decode weights matter):

* engine  — the decode engine (prefill + eager decode steps of ``CausalLM.decode``: the fused
  GEMV layer at batch <= 16, the 256x128 split-K layer at batch > 64), per-layer residual stream
  captured at every decode step;
* train   — the training / scoring forward (``CausalLM.forward``, 256x256 MFMA GEMMs, flash
  attention) over [prompt | generated tokens], residual stream at the same positions;
* fp32    — the same weights (bf16-rounded, merged LoRA) in fp32 on the CPU (eager oracles).

Printed per layer: relative L2 error of engine vs fp32, train vs fp32, engine vs train, and the
final log-prob gap of the sampled tokens. Usage (GPU box):
  python tools/r6/divergence_trace.py --batch 1 --steps 24
  python tools/r6/divergence_trace.py --batch 256 --steps 16 --oracle-rows 2
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--prompt", type=int, default=173)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--lora", type=float, default=0.02, help="std of the LoRA A / B draws (0: no adapters)")
    ap.add_argument("--oracle-rows", type=int, default=1, help="rows scored by the fp32 CPU oracle")
    args = ap.parse_args()

    from rag_tl_domainllm_optimizer_amd import models, ops
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models.decoder import CausalLM, DecoderLayer, fast_random_init_
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    dev = torch.device("cuda:0")
    cfg = dataclasses.replace(models.resolve_preset("mistral-7b"), num_layers=args.layers, name="mistral-7b-width")
    m = CausalLM(cfg, device=dev, dtype=torch.bfloat16, init=False)
    fast_random_init_(m, seed=3)
    if args.lora > 0:
        m.add_lora(16, 32.0, None, seed=5)
        with torch.no_grad():
            g = torch.Generator(device=dev).manual_seed(9)
            for p in m.lora_parameters():
                p.normal_(0.0, args.lora, generator=g)
        m.refresh_lora()
    B, T = args.batch, args.steps + 1
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(5, cfg.vocab_size, (args.prompt,), generator=g).tolist() for _ in range(B)]

    # ---- engine: prefill + eager decode steps, residual stream per layer per step ----
    cap = {"on": False, "layers": [], "steps": []}
    orig_fused, orig_mlp = DecoderLayer.decode_fused, DecoderLayer.mlp

    def fused(self, h, attend):
        out = orig_fused(self, h, attend)
        if cap["on"]:
            cap["layers"].append(out.detach().clone())
        return out

    def mlp(self, a, residual, defer=False):
        x, res = orig_mlp(self, a, residual, defer)
        if cap["on"] and not torch.is_grad_enabled():
            xs = x.reduce() if isinstance(x, ops.SplitK) else x
            cap["layers"].append((xs.float() + res.float()).to(torch.bfloat16).detach().clone())
        return x, res

    orig_decode = CausalLM.decode

    def decode(self, *a, **k):
        cap["on"], cap["layers"] = True, []
        y = orig_decode(self, *a, **k)
        cap["on"] = False
        cap["steps"].append(cap["layers"])
        return y

    DecoderLayer.decode_fused, DecoderLayer.mlp, CausalLM.decode = fused, mlp, decode
    try:
        gen = Generator(m, B, args.prompt + T + 8, dev, use_graph=False)
        out = gen.generate(prompts, SamplingParams(max_new_tokens=T, temperature=0.7, top_k=50, seed=7), pad_id=0,
                           eos_ids=[-1])
    finally:
        DecoderLayer.decode_fused, DecoderLayer.mlp, CausalLM.decode = orig_fused, orig_mlp, orig_decode
    steps = cap["steps"]  # decode call i (token i fed at position S + i) -> residual streams [B, H] per layer
    path = "fused GEMV layer (batch <= 16)" if B <= m.fused_decode_max_batch else "split-K 256x128 layer (batch > 64)"
    print(f"# {cfg.num_layers}-layer Mistral-7B-width, batch {B} ({path}), prompt {args.prompt}, {len(steps)} decode "
          f"steps, LoRA std {args.lora}")

    # ---- train: the scoring forward over [prompt | tokens], same capture ----
    seq = torch.cat([out.prompt_ids, out.tokens], 1)
    S = out.prompt_ids.shape[1]
    tcap = []
    orig_layer_fwd = CausalLM._layer_fwd

    def layer_fwd(self, layer, x, residual, *a, **k):
        xo, ro = orig_layer_fwd(self, layer, x, residual, *a, **k)
        tcap.append((xo.float() + ro.float()).to(torch.bfloat16).detach())
        return xo, ro

    CausalLM._layer_fwd = layer_fwd
    try:
        with torch.no_grad():
            m(seq, kv_start=out.prompt_start.to(torch.int32))
        m_tcap = list(tcap)
        tcap.clear()
    finally:
        CausalLM._layer_fwd = orig_layer_fwd
    L = seq.shape[1]
    with torch.no_grad():
        lp_train, _, _, _ = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)

    # ---- fp32 CPU oracle on the first rows: merged bf16 weights, eager reference ops ----
    R = min(args.oracle_rows, B)
    cpu = CausalLM(cfg, device="cpu", dtype=torch.float32, init=False)
    with torch.no_grad():
        prev = m.set_lora_merged(True)
        sd = {}
        for name, p in m.named_parameters():
            if "lora" in name:
                continue
            sd[name] = p.detach()
        for li, layer in enumerate(m.layers):
            for gname, wname in (("qkv", "qkv_w"), ("o", "o_w"), ("gate_up", "gate_up_w"), ("down", "down_w")):
                grp = layer.lora.get(gname)
                if grp is not None:
                    sd[f"layers.{li}.{wname}"] = grp.merged_weight(getattr(layer, wname)).detach()
        m.set_lora_merged(prev)
        for name, p in cpu.named_parameters():
            p.copy_(sd[name].float().cpu())
    ocap = []

    def oracle_layer_fwd(self, layer, x, residual, *a, **k):
        xo, ro = orig_layer_fwd(self, layer, x, residual, *a, **k)
        ocap.append((xo.float() + ro.float()).detach())
        return xo, ro

    CausalLM._layer_fwd = oracle_layer_fwd
    try:
        with torch.no_grad():
            cpu(seq[:R].cpu(), kv_start=out.prompt_start[:R].to(torch.int32).cpu())
    finally:
        CausalLM._layer_fwd = orig_layer_fwd

    # ---- compare at the decoded positions of the oracle rows ----
    print("layer  engine_vs_fp32  train_vs_fp32  engine_vs_train   (relative L2 over the decode steps, rows "
          f"0..{R - 1}; engine_vs_train also over all {B} rows: see last column)")
    for li in range(cfg.num_layers):
        e, t, o, e_all, t_all = [], [], [], [], []
        for j in range(len(steps)):
            p = S + j
            e.append(steps[j][li][:R].float().cpu())
            t.append(m_tcap[li].view(B, L, -1)[:R, p].float().cpu())
            o.append(ocap[li].view(R, L, -1)[:, p])
            e_all.append(steps[j][li].float())
            t_all.append(m_tcap[li].view(B, L, -1)[:, p].float())
        e, t, o = torch.stack(e), torch.stack(t), torch.stack(o)
        print(f"{li:5d}  {rel(e, o):14.3e}  {rel(t, o):13.3e}  {rel(e, t):15.3e}   all rows {rel(torch.stack(e_all), torch.stack(t_all)):.3e}")
    mask = torch.arange(T, device=dev)[None] < out.lengths[:, None]
    gap = ((lp_train - out.logprobs).abs() * mask).sum() / mask.sum()
    print(f"sampled-token log-prob gap |engine - train|: {float(gap):.3e} nats/token (mean), "
          f"max {float(((lp_train - out.logprobs).abs() * mask).max()):.3e}")


if __name__ == "__main__":
    main()
