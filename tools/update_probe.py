"""Is the PPO update launch-bound? Times one update() (4 minibatches of 16 x 448 tokens,
Mistral-7B shape, LoRA r=16) three ways: host issue time of each stage (no sync), GPU time of each
stage (events), and wall time. A stage whose host issue time exceeds its GPU time starves the GPU.

    python tools/update_probe.py [--model mistral-7b] [--mb 16] [--prompt 320] [--resp 128]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--mb", type=int, default=16)
    ap.add_argument("--prompt", type=int, default=320)
    ap.add_argument("--resp", type=int, default=128)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--cprofile", action="store_true", help="host-side cProfile of the measured iterations")
    ap.add_argument("--torch-prof", action="store_true", help="torch.profiler op table grouped by input shape")
    ap.add_argument("--trainer", action="store_true",
                    help="time PPOTrainer.update() on a synthetic 64-sequence rollout (wall vs GPU-only)")
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd import ops
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.models.value_head import ValueHead
    from rag_tl_domainllm_optimizer_amd.train.common import masked_mean, score_sequences

    dev = torch.device("cuda")
    if a.trainer:
        return trainer_probe(a, dev)
    pol = build_model(a.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    pol.add_lora(16, 32.0, ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"], seed=0)
    pol.freeze_base()
    vh = ValueHead(pol.cfg.hidden_size, device=dev, seed=1)
    flat = ops.FlatParams(list(pol.lora_parameters()) + list(vh.parameters()))
    pol.refresh_lora()
    opt = ops.FusedAdamW(flat, lr=1e-5)
    B, S, T = a.mb, a.prompt, a.resp
    V = pol.cfg.vocab_size
    prompt = torch.randint(5, V, (B, S), device=dev)
    start = torch.randint(0, S // 4, (B,), device=dev)
    resp = torch.randint(5, V, (B, T), device=dev)
    rlen = torch.randint(T // 2, T + 1, (B,), device=dev)
    old = torch.randn(B, T, device=dev) * 0.1 - 2
    adv = torch.randn(B, T, device=dev)

    def step(marks):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t = [time.perf_counter()]
        ev[0].record()
        lp, ent, vals, mask = score_sequences(pol, prompt, start, resp, rlen, 1 / 0.7, vh, False)
        ratio = torch.exp(lp - old)
        loss = masked_mean(-torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv), mask) + \
            0.5 * masked_mean(vals ** 2, mask) - 0.01 * masked_mean(ent, mask)
        t.append(time.perf_counter())
        ev[1].record()
        opt.zero_grad()
        loss.backward()
        t.append(time.perf_counter())
        ev[2].record()
        opt.step(1e-5)
        pol.refresh_lora()
        t.append(time.perf_counter())
        ev[3].record()
        marks.append((t, ev))

    for _ in range(2):
        step([])
    torch.cuda.synchronize()
    marks = []
    prof = None
    if a.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    w0 = time.perf_counter()
    for _ in range(a.iters):
        step(marks)
    torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(35)
    wall = (time.perf_counter() - w0) / a.iters
    names = ["forward", "backward", "optimizer"]
    host = [sum(m[0][i + 1] - m[0][i] for m in marks) / a.iters * 1e3 for i in range(3)]
    gpu = [sum(m[1][i].elapsed_time(m[1][i + 1]) for m in marks) / a.iters for i in range(3)]
    print(f"minibatch {B}x{S + T} tokens: wall {wall * 1e3:.1f} ms")
    for n, h, g in zip(names, host, gpu):
        print(f"  {n:10s} host issue {h:8.1f} ms   gpu {g:8.1f} ms")
    if a.torch_prof:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as tp:
            step([])
            torch.cuda.synchronize()
        print(tp.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45,
                                                                 max_name_column_width=40, max_shapes_column_width=70))
    # pure-GPU time with the host out of the way: replay the same step after a long queue
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2e9))  # ~1 s of queued work so the host runs ahead
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    step([])
    e1.record()
    torch.cuda.synchronize()
    print(f"  GPU-only (host ahead) step: {e0.elapsed_time(e1):.1f} ms")


def trainer_probe(a, dev):
    from rag_tl_domainllm_optimizer_amd.models import build_model
    from rag_tl_domainllm_optimizer_amd.train.ppo import PPOConfig, PPOTrainer, Rollout

    pol = build_model(a.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    pc = PPOConfig(max_new_tokens=a.resp, max_prompt_tokens=a.prompt, minibatch_size=a.mb, lora_r=16,
                   lora_alpha=32.0, seed=0)
    tr = PPOTrainer(pol, None, None, pc, max_batch=64)
    B, S, T, V = 64, a.prompt, a.resp, pol.cfg.vocab_size
    g = torch.Generator(device="cpu").manual_seed(0)
    ro = Rollout(prompt_ids=torch.randint(5, V, (B, S), generator=g).to(dev),
                 start=torch.randint(0, S // 3, (B,), generator=g).to(dev),
                 resp=torch.randint(5, V, (B, T), generator=g).to(dev),
                 resp_len=torch.randint(T // 2, T + 1, (B,), generator=g).to(dev),
                 old_logp=(torch.randn(B, T, generator=g) * 0.1 - 2).to(dev),
                 old_values=torch.randn(B, T, generator=g).to(dev), scores=torch.zeros(B, device=dev),
                 components={}, responses=[], queries=[])
    ro.adv = torch.randn(B, T, device=dev)
    ro.returns = torch.randn(B, T, device=dev)
    for _ in range(2):
        tr.update(ro)
    torch.cuda.synchronize()
    walls = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        tr.update(ro)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
    torch.cuda._sleep(int(4e9))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    upd = tr.update  # host issues everything while the GPU sleeps (the final float() waits)
    upd(ro)
    e1.record()
    torch.cuda.synchronize()
    print(f"trainer.update (64 seq, mb {a.mb}): wall {min(walls) * 1e3:.1f} ms; GPU-only {e0.elapsed_time(e1):.1f} ms "
          "(GPU-only includes the sleep if the host could not get ahead)")


if __name__ == "__main__":
    main()
