"""Behaviour / target policy gap of PPO rollouts: rollouts (prefill + decode, sampler
log-probs at temperature 0.7) vs the training forward's scoring of the same tokens at the same
weights (theta = theta_old), on a random-init model with LoRA adapters of a given magnitude.

    python tools/r5/behaviour_gap_probe.py [--model tiny-mistral] [--batch 8] [--new 16]

Prints mean |logp_score - logp_rollout| (nats / token) for merged-bf16 rollouts and for rollouts on
the unmerged LoRA K-extension, per adapter scale (B ~ N(0, sigma); sigma 0 = no adapter delta).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tiny-mistral")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=40)
    ap.add_argument("--new", type=int, default=16)
    ap.add_argument("--sigmas", default="0,1e-4,1e-3")
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd import models, ops
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    ops.native()
    dev = torch.device("cuda")
    m = build_model(a.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    m.add_lora(16, 32.0, "all")
    m.freeze_base()
    cfg = m.cfg
    g = torch.Generator(device="cpu").manual_seed(5)
    prompts = [torch.randint(3, cfg.vocab_size, (a.prompt - (i % 3),), generator=g).tolist() for i in range(a.batch)]
    gen = Generator(m, a.batch, a.prompt + a.new + 8, dev)
    for sigma in [float(s) for s in a.sigmas.split(",")]:
        with torch.no_grad():
            for n, p in m.named_parameters():
                if "lora" in n and n.endswith("_B"):
                    p.normal_(0, sigma) if sigma > 0 else p.zero_()
        m.refresh_lora()
        for merged in (True, False):
            gen.merge_lora = merged
            torch.manual_seed(11)
            out = gen.generate(prompts, SamplingParams(max_new_tokens=a.new, temperature=0.7, top_k=50, do_sample=True,
                                                       seed=3), pad_id=0, eos_ids=[-1])
            with torch.no_grad():
                lp, _, _, mask = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths,
                                                 1.0 / 0.7)
            mf = mask.float()
            d = (lp.float() - out.logprobs.float()).abs() * mf
            gap = float(d.sum() / mf.sum())
            print(f"{a.model} sigma={sigma:g} merged={merged}: mean |dlogp| = {gap:.3e} nats/token, "
                  f"max {float(d.max()):.3e}, mean logp {float((lp * mf).sum() / mf.sum()):.3f}", flush=True)


if __name__ == "__main__":
    main()
