"""One rollout-shaped generation (Mistral-7B, random init, LoRA r=16 merged) for kernel profiling:
    rocprofv3 --kernel-trace --stats -- python tools/decode_profile.py --batch 64 --new 64
Prints the per-step wall time; the rocprof stats give the per-kernel split of a decode step."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=300)
    ap.add_argument("--new", type=int, default=64)
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--no-lora", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="fp8 weight images (config 5)")
    ap.add_argument("--fp8-kv", action="store_true", help="fp8 K/V cache (config 5)")
    ap.add_argument("--depths", default="0", help="M<=16 GEMM weight-pipeline depths to A/B (0 = auto)")
    ap.add_argument("--iters", type=int, default=3, help="generations per depth")
    ap.add_argument("--no-graph", action="store_true", help="eager decode steps (counter collection)")
    ap.add_argument("--fused-max", type=int, default=-1, help="bf16 fused decode layer up to this batch (-1: model default)")
    ap.add_argument("--set", default="", help="native tuning knobs for the run, k=v[,k=v]")
    a = ap.parse_args()
    from rag_tl_domainllm_optimizer_amd.generation import Generator, SamplingParams
    from rag_tl_domainllm_optimizer_amd.models import build_model

    dev = torch.device("cuda")
    if a.set:
        from rag_tl_domainllm_optimizer_amd import ops as _ops

        _ops.native().set_tuning({k: int(v) for k, v in (kv.split("=") for kv in a.set.split(","))})
    m = build_model(a.model, device=dev, dtype=torch.bfloat16, seed=0, fast_init=True)
    if not a.no_lora:
        m.add_lora(16, 32.0, "all")
    if a.fp8:
        m.set_fp8(True)
    if a.fused_max >= 0:
        m.fused_decode_max_batch = a.fused_max
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(5, m.cfg.vocab_size, (a.prompt - (i % 7) * 3,), generator=g).tolist()
               for i in range(a.batch)]
    gen = Generator(m, a.batch, a.prompt + a.new + 8, dev, kv_fp8=a.fp8_kv, use_graph=not a.no_graph)
    sp = SamplingParams(max_new_tokens=a.new, temperature=0.7, top_k=50)
    from rag_tl_domainllm_optimizer_amd import ops

    for it, depth in enumerate([int(d) for d in a.depths.split(",") for _ in range(a.iters)]):
        ops.native().set_tuning({"decode_depth": depth})
        if it % a.iters == 0 and gen.use_graph:
            gen.runner.reset()  # the launch choice is baked into the captured decode graph
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = gen.generate_async(prompts, sp, pad_id=0, eos_ids=[-1]).result()
        dt = time.perf_counter() - t0
        print(f"iter {it} depth {depth}: total {dt * 1e3:.1f} ms prefill {out.timings['prefill_s'] * 1e3:.1f} ms decode "
              f"{out.timings['decode_s'] * 1e3:.1f} ms = {out.timings['decode_s'] / (a.new - 1) * 1e3:.3f} ms/step",
              flush=True)


if __name__ == "__main__":
    main()
