"""Config-5 decode path A/B on Llama-2-13B shape (random init, fp8 weights + fp8 K/V): one batch-256
rollout (173-token prompts, 128 new tokens, temperature 0.7, top-k 50) with the W8A8 split-K
partials deferred to the norms / attention prologue vs reduced eagerly: generated tokens (EOS
early exits), agreement, and the mean |log-prob| gap to a teacher-forced rescoring.

    python tools/r5/fp8_defer_probe.py [--batch 256]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-13b")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--new", type=int, default=128)
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.train.common import score_sequences

    dev = torch.device("cuda")
    model = build_model(a.model + ":random", device=dev, fast_init=True)
    model.set_fp8(True)
    cfg = model.cfg
    eos = cfg.eos_token_id
    g = torch.Generator(device="cpu").manual_seed(1)
    prompts = torch.randint(5, cfg.vocab_size, (a.batch, 173), generator=g).tolist()
    p = SamplingParams(max_new_tokens=a.new, temperature=0.7, top_k=50, seed=7)
    for defer in (False, True, False, True):
        model.defer_splitk = defer
        gen = Generator(model, a.batch, 173 + a.new + 8, dev, kv_fp8=True)
        torch.cuda.synchronize()
        t0 = time.time()
        out = gen.generate(prompts, p, pad_id=0, eos_ids=[eos])
        torch.cuda.synchronize()
        el = time.time() - t0
        n = int(out.lengths.sum())
        with torch.no_grad():
            lp, _, _, _ = score_sequences(model, out.prompt_ids, out.prompt_start, out.tokens, out.lengths, 1 / 0.7)
        mask = torch.arange(out.tokens.shape[1], device=dev)[None, :] < out.lengths[:, None]
        gap = ((lp - out.logprobs).abs() * mask).sum() / mask.sum()
        first_eos = (out.tokens == eos).float().argmax(1)
        print(f"defer={defer}: {el:.2f}s tokens={n} ({n / (a.batch * a.new):.3f} of max) rows_with_eos="
              f"{int((out.tokens == eos).any(1).sum())} teacher-forced gap={gap.item():.4f}", flush=True)
        del gen


if __name__ == "__main__":
    main()
