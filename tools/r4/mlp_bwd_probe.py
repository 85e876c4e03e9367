"""Training MLP (Mistral-7B shapes, LoRA r=16 on gate / up / down) forward + backward at M = 9632
tokens: the fused node (ops.swiglu_mlp: SwiGLU backward in the down dX GEMM epilogue) vs the two
linears (separate swiglu_bwd pass), interleaved rounds on one device."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import models, ops  # noqa: E402


def main():
    cfg = models.resolve_preset("mistral-7b")
    dev = "cuda"
    H, F = cfg.hidden_size, cfg.intermediate_size
    w_gu = (torch.randn(2 * F, H, device=dev) * 0.02).to(torch.bfloat16)
    w_d = (torch.randn(H, F, device=dev) * 0.02).to(torch.bfloat16)

    def group(n_out, K, rows, seed):
        g = torch.Generator(device="cpu").manual_seed(seed)
        a = [torch.nn.Parameter((torch.randn(16, K, generator=g) * 0.02).to(dev)) for _ in rows]
        b = [torch.nn.Parameter((torch.randn(n, 16, generator=g) * 0.02).to(dev)) for n in rows]
        c0 = [0] + [sum(rows[:i + 1]) for i in range(len(rows) - 1)]
        grp = ops.LoRAGroup(["p"] * len(rows), a, b, c0, [2.0] * len(rows), n_out)
        grp.refresh()
        return grp

    lg, ld = group(2 * F, H, [F, F], 1), group(H, F, [H], 2)
    M = 9632
    x = (torch.randn(M, H, device=dev)).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(M, H, device=dev).to(torch.bfloat16)

    def fused():
        y = ops.swiglu_mlp(x, w_gu, w_d, lg, ld)
        y.backward(gy)

    def unfused():
        f = ops.linear(x, w_gu, act="swiglu", lora=lg)
        y = ops.linear(f, w_d, lora=ld)
        y.backward(gy)

    def timeit(fn, iters=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters

    res = {"fused": [], "unfused": []}
    for _ in range(5):
        res["fused"].append(timeit(fused))
        res["unfused"].append(timeit(unfused))
    for k, v in res.items():
        print(f"{k}: {statistics.median(v):.3f} ms per MLP fwd+bwd (min {min(v):.3f})", flush=True)


if __name__ == "__main__":
    main()
