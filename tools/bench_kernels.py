"""Microbenchmarks of the hand-written kernels vs the library equivalents on Mistral-7B shapes.

Usage: python tools/bench_kernels.py [--json out.json]
Prints one line per case: time (us), achieved TFLOP/s or GB/s, and the library reference time.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = "cuda"
    res = []
    H, F, NQKV, V = 4096, 14336, 6144, 32000
    gemms = [("qkv", NQKV, H), ("o", H, H), ("gate_up", 2 * F, H), ("down", H, F), ("lm_head", V, H)]
    for M in (1, 16, 64, 2048, 8192):
        for name, N, K in gemms:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            t_ours = timeit(lambda: ops.gemm(a, w))
            t_lib = timeit(lambda: a @ w.t())
            flops = 2 * M * N * K
            byts = 2 * (N * K + M * K + M * N)
            r = dict(kind="gemm", name=name, M=M, N=N, K=K, us=t_ours, lib_us=t_lib,
                     tflops=flops / t_ours / 1e6, lib_tflops=flops / t_lib / 1e6, gbs=byts / t_ours / 1e3)
            res.append(r)
            print(json.dumps(r), flush=True)
    # LoRA-fused vs separate
    for M in (2048, 8192):
        N, K, R = NQKV, H, 64
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        ap_ = torch.randn(R, K, device=dev, dtype=torch.bfloat16)
        ub = torch.randn(N, R, device=dev, dtype=torch.bfloat16)
        t_f = timeit(lambda: ops.gemm(a, w, ops.gemm(a, ap_), ub))
        t_l = timeit(lambda: a @ w.t() + (a @ ap_.t()) @ ub.t())
        r = dict(kind="gemm_lora", M=M, N=N, K=K, us=t_f, lib_us=t_l)
        res.append(r)
        print(json.dumps(r), flush=True)
    # attention prefill fwd
    for B, S in ((16, 384), (4, 2048)):
        Hq, Hkv, D = 32, 8, 128
        qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hkv, D, True))
        q = qkv[:, :Hq * D].reshape(B, S, Hq, D).transpose(1, 2)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(4, 1)
        v = qkv[:, (Hq + Hkv) * D:].reshape(B, S, Hkv, D).transpose(1, 2).repeat_interleave(4, 1)
        tl = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True))
        flops = 4 * B * Hq * S * S * D / 2
        r = dict(kind="attn_fwd", B=B, S=S, us=t, lib_us=tl, tflops=flops / t / 1e6, lib_tflops=flops / tl / 1e6)
        res.append(r)
        print(json.dumps(r), flush=True)
        x = qkv.clone().requires_grad_(True)
        o = ops.flash_attention_qkv(x, B, S, Hq, Hkv, D, True)
        go = torch.randn_like(o)
        t = timeit(lambda: torch.autograd.grad(o, x, go, retain_graph=True), iters=10)
        r = dict(kind="attn_bwd", B=B, S=S, us=t, tflops=2.5 * flops / t / 1e6)
        res.append(r)
        print(json.dumps(r), flush=True)
    # decode attention
    for B, L in ((1, 512), (64, 512), (64, 2048)):
        Hq, Hkv, D = 32, 8, 128
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        kc = torch.randn(B, Hkv, L, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        lens = torch.full((B,), L, device=dev, dtype=torch.int32)
        ws = ops.decode_workspace(B, Hq, Hkv, D, L, dev)
        out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: ops.decode_attention(q, kc, vc, lens, Hq, workspace=ws, out=out))
        byts = 2 * kc.numel() * 2
        r = dict(kind="attn_decode", B=B, L=L, us=t, gbs=byts / t / 1e3)
        res.append(r)
        print(json.dumps(r), flush=True)
    # norm / logprob / sampler
    x = torch.randn(8192, H, device=dev, dtype=torch.bfloat16)
    rr = torch.randn_like(x)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.rms_norm(x, w, 1e-5, rr))
    r = dict(kind="add_rmsnorm", T=8192, us=t, gbs=4 * x.numel() * 2 / t / 1e3)
    res.append(r)
    print(json.dumps(r), flush=True)
    logits = torch.randn(8192, V, device=dev, dtype=torch.bfloat16)
    tgt = torch.randint(0, V, (8192,), device=dev)
    t = timeit(lambda: ops.token_logprobs(logits, tgt, 1.0))
    r = dict(kind="logprob", T=8192, us=t, gbs=logits.numel() * 2 / t / 1e3)
    res.append(r)
    print(json.dumps(r), flush=True)
    lg = torch.randn(64, V, device=dev, dtype=torch.bfloat16)
    off = torch.zeros(1, dtype=torch.long, device=dev)
    t = timeit(lambda: ops.sample(lg, 1 / 0.7, top_k=50, top_p=0.9, seed=1, offset=off))
    r = dict(kind="sample_topk_topp", B=64, us=t)
    res.append(r)
    print(json.dumps(r), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
