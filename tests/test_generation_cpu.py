"""Generation engine on CPU: KV-cache decode == no-cache recompute (greedy), stop handling."""
import pytest
import torch

from rag_tl_domainllm_optimizer_amd import models
from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS


def _greedy_ref(model, prompt, n):
    ids = list(prompt)
    out = []
    for _ in range(n):
        with torch.no_grad():
            h = model(torch.tensor([ids]))
            nxt = int(model.logits(h[-1:]).argmax(-1))
        out.append(nxt)
        ids.append(nxt)
    return out


def test_kv_cache_greedy_matches_recompute():
    for preset in ("tiny-llama", "tiny-mistral", "tiny-opt"):
        cfg = PRESETS[preset]
        m = models.CausalLM(cfg, dtype=torch.float32, seed=3)
        prompts = [[5, 9, 33, 41, 7], [12, 300, 4], [77] * 9]
        gen = Generator(m, max_batch=4, max_seq=32, device="cpu")
        out = gen.generate(prompts, SamplingParams(max_new_tokens=6, do_sample=False), pad_id=0, eos_ids=[-5])
        for b, p in enumerate(prompts):
            assert out.tokens[b].tolist() == _greedy_ref(m, p, 6), (preset, b)
            assert int(out.lengths[b]) == 6


def test_eos_stops_row():
    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=3)
    prompts = [[5, 9, 33, 41, 7]]
    ref = _greedy_ref(m, prompts[0], 6)
    gen = Generator(m, max_batch=2, max_seq=32, device="cpu")
    out = gen.generate(prompts, SamplingParams(max_new_tokens=6, do_sample=False), pad_id=0, eos_ids=[ref[2]])
    assert int(out.lengths[0]) == 3
    assert out.tokens[0, :3].tolist() == ref[:3]


def test_sampling_logprobs_consistent():
    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=3)
    torch.manual_seed(0)
    gen = Generator(m, max_batch=2, max_seq=40, device="cpu")
    prompts = [[5, 9, 33], [8, 8]]
    p = SamplingParams(max_new_tokens=5, temperature=0.7, top_k=0)
    out = gen.generate(prompts, p, pad_id=0, eos_ids=[-1])
    # behaviour log-probs equal a teacher-forced recompute of the same tokens
    for b, pr in enumerate(prompts):
        seq = pr + out.tokens[b].tolist()
        with torch.no_grad():
            lg = m.logits(m(torch.tensor([seq])))
        lp = torch.log_softmax(lg.float() / 0.7, -1)
        exp = [lp[len(pr) - 1 + t, seq[len(pr) + t]].item() for t in range(5)]
        torch.testing.assert_close(out.logprobs[b], torch.tensor(exp), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("k", [3, 9, 21])
def test_async_early_exit_matches_full_run(k):
    """Rollouts stop once every row has emitted EOS ("async" early exit: flags read behind events,
    two chunks ahead). Forcing EOS at step k (EOS ids = the tokens each row drew at step k) ends
    the loop after ~k steps, with outputs and the sampler's RNG counter identical to the run that
    enqueues every step."""
    from rag_tl_domainllm_optimizer_amd import models
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models.config import PRESETS

    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=3)
    prompts = [list(range(5, 25)), list(range(9, 40)), list(range(30, 36))]
    sp = SamplingParams(max_new_tokens=40, temperature=0.7, top_k=20, seed=5)
    g = Generator(m, 3, 100, sync_every=4)
    torch.manual_seed(0)  # the CPU sampler draws from the global generator (the GPU one: Philox offsets)
    full = g.generate_async(prompts, sp, pad_id=0, eos_ids=[-1]).result()
    eos = sorted({int(t) for t in full.tokens[:, k].tolist()})
    g.rng_offset.zero_()
    torch.manual_seed(0)
    ref = g.generate_async(prompts, sp, pad_id=0, eos_ids=eos).result()
    off_ref = int(g.rng_offset)
    g.rng_offset.zero_()
    torch.manual_seed(0)
    h = g.generate_async(prompts, sp, pad_id=0, eos_ids=eos, early_stop="async")
    out = h.result()
    assert torch.equal(out.tokens, ref.tokens) and torch.equal(out.lengths, ref.lengths)
    assert torch.equal(out.logprobs, ref.logprobs)
    assert int(g.rng_offset) == off_ref  # skipped steps still advance the RNG counter
    assert int(out.lengths.max()) <= k + 1
    # the loop ran at most the chunks up to step k plus the two chunks kept ahead
    assert out.timings["decode_steps"] <= min(39, (k // 4 + 3) * 4)
    assert out.timings["decode_steps"] < 39 or k >= 30
