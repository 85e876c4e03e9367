"""Where the behaviour / target gap of PPO rollouts comes from at Mistral-7B shape (random init,
bf16, LoRA r16 all linear with a trained-size B): sampler log-probs of generated tokens vs the
training forward's scoring of the same tokens (theta = theta_old), per batch size (decode kernel
regime) and response position, plus the signed mean (a systematic bias points at a bug, noise at
kernel numerics).

    python tools/r5/behaviour_gap_7b.py [--batches 8,96,256] [--new 32]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--batches", default="8,96,256")
    ap.add_argument("--prompt", type=int, default=173)
    ap.add_argument("--new", type=int, default=32)
    ap.add_argument("--sigma", type=float, default=3e-4)
    ap.add_argument("--temp", type=float, default=0.7)
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd import ops
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    ops.native()
    dev = torch.device("cuda")
    m = build_model(a.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    m.add_lora(16, 32.0, "all")
    m.freeze_base()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "lora" in n and n.endswith("_B"):
                p.normal_(0, a.sigma)
    m.refresh_lora()
    cfg = m.cfg
    bmax = max(int(b) for b in a.batches.split(","))
    g = torch.Generator(device="cpu").manual_seed(5)
    prompts = [torch.randint(3, cfg.vocab_size, (a.prompt - (i % 7),), generator=g).tolist() for i in range(bmax)]
    gen = Generator(m, bmax, a.prompt + a.new + 8, dev)
    for B in [int(b) for b in a.batches.split(",")]:
        for merged in (True, False):
            gen.merge_lora = merged
            out = gen.generate(prompts[:B], SamplingParams(max_new_tokens=a.new, temperature=a.temp, top_k=50,
                                                           do_sample=True, seed=3), pad_id=0, eos_ids=[-1])
            with torch.no_grad():
                lp, _, _, mask = score_sequences(m, out.prompt_ids, out.prompt_start, out.tokens, out.lengths,
                                                 1.0 / a.temp)
                # greedy-free check of the prompt part: the training forward's logp of the FIRST
                # generated token vs the prefill's (no decode step involved)
            mf = mask.float()
            d = (lp.float() - out.logprobs.float()) * mf
            n = mf.sum()
            per_t = (d.abs().sum(0) / mf.sum(0).clamp(min=1)).tolist()
            print(f"B={B:3d} merged={merged}: mean|d| {float(d.abs().sum() / n):.4f}  mean d {float(d.sum() / n):+.4f}  "
                  f"max|d| {float(d.abs().max()):.3f}  mean logp {float((lp * mf).sum() / n):.3f}", flush=True)
            print("   |d| by position: " + " ".join(f"{x:.3f}" for x in per_t[:: max(1, len(per_t) // 16)]), flush=True)


if __name__ == "__main__":
    main()
