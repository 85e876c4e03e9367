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
    ap.add_argument("--only", default=None, help="comma list of kinds: gemm,lora,attn,decode,norm,loss,sample")
    args = ap.parse_args()
    only = set(args.only.split(",")) if args.only else None

    def want(k):
        return only is None or k in only

    pass  # single (hand-written) GEMM path since round 2
    C = ops.native()
    dev = "cuda"
    res = []
    H, F, NQKV, V = 4096, 14336, 6144, 32000
    gemms = [("qkv", NQKV, H), ("o", H, H), ("gate_up", 2 * F, H), ("down", H, F), ("lm_head", V, H)]
    for M in (1, 16, 64, 512, 2048, 7168, 20480):
        if not want("gemm"):
            break
        for name, N, K in gemms:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) / math.sqrt(K)
            t_lib = timeit(lambda: a @ w.t())
            flops = 2 * M * N * K
            byts = 2 * (N * K + M * K + M * N)
            variants = [("auto", 0)] if M <= 64 else [("t128", 1), ("t256", 2), ("auto", 0)]
            for vname, v in variants:
                C.set_tuning({"gemm_variant": v})
                t_ours = timeit(lambda: ops.gemm(a, w))
                r = dict(kind="gemm", variant=vname, name=name, M=M, N=N, K=K, us=t_ours, lib_us=t_lib,
                         tflops=flops / t_ours / 1e6, lib_tflops=flops / t_lib / 1e6, gbs=byts / t_ours / 1e3)
                res.append(r)
                print(json.dumps(r), flush=True)
            C.set_tuning({"gemm_variant": 0})
    # skinny GEMMs with the weights streamed from HBM (rotating copies > the 256 MB Infinity
    # Cache), which is what a decode step sees
    for M in ((1, 8, 32, 64) if want("cold") else ()):
        for name, N, K in gemms:
            ncopy = max(2, int(1.2e9 // (N * K * 2)))
            ws_ = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) / math.sqrt(K) for _ in range(ncopy)]
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            it = [0]

            def run(fn):
                it[0] = (it[0] + 1) % ncopy
                return fn(ws_[it[0]])

            t_n = timeit(lambda: run(lambda w_: ops.gemm(a, w_)), iters=ncopy * 2)
            t_l = timeit(lambda: run(lambda w_: a @ w_.t()), iters=ncopy * 2)
            byts = 2 * N * K
            r = dict(kind="gemm_cold", name=name, M=M, N=N, K=K, us=t_n, lib_us=t_l, gbs=byts / t_n / 1e3,
                     lib_gbs=byts / t_l / 1e3)
            res.append(r)
            print(json.dumps(r), flush=True)
            del ws_
        torch.cuda.empty_cache()
    # fp8: W8A8 MX-MFMA tile kernel (large M, incl. per-token activation quantisation) and W8A16
    # skinny decode (cold weights)
    for M in ((7168, 20480) if want("fp8") else ()):
        for name, N, K in gemms:
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16)
            wq, sw = ops.quantize_fp8(w)
            xq, sx = ops.quantize_fp8(a)
            t8 = timeit(lambda: C.gemm_fp8(xq, sx, wq, sw))
            tq = timeit(lambda: ops.quantize_fp8(a))
            tl = timeit(lambda: a @ w.t())
            flops = 2 * M * N * K
            r = dict(kind="gemm_fp8", name=name, M=M, N=N, K=K, us=t8, quant_us=tq, bf16_lib_us=tl,
                     tflops=flops / t8 / 1e6, tflops_with_quant=flops / (t8 + tq) / 1e6, lib_tflops=flops / tl / 1e6)
            res.append(r)
            print(json.dumps(r), flush=True)
    for M in ((1, 16, 64) if want("fp8") else ()):
        for name, N, K in gemms:
            ncopy = max(2, int(1.2e9 // (N * K)))
            wqs = [ops.quantize_fp8((torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16))
                   for _ in range(ncopy)]
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            it = [0]

            def run8():
                it[0] = (it[0] + 1) % ncopy
                return C.gemm_fp8(a, None, wqs[it[0]][0], wqs[it[0]][1])

            t8 = timeit(run8, iters=ncopy * 2)
            r = dict(kind="gemm_w8a16_cold", name=name, M=M, N=N, K=K, us=t8, gbs=N * K / t8 / 1e3)
            res.append(r)
            print(json.dumps(r), flush=True)
            del wqs
        torch.cuda.empty_cache()
    # fused decode attention at batch 1: partition size sweep (NP = ceil(Smax / PS))
    for L in ((456, 2048) if want("attnps") else ()):
        Hq, Hkv, D = 32, 8, 128
        q1 = torch.randn(1, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        kc1 = torch.randn(1, Hkv, L + 8, D, device=dev, dtype=torch.bfloat16)
        vc1 = torch.randn_like(kc1)
        slot = torch.full((1,), L - 1, device=dev, dtype=torch.int32)
        cos, sin = ops.reference.rope_tables(D, 8192, 10000.0, dev)
        o1 = torch.empty(1, Hq * D, device=dev, dtype=torch.bfloat16)
        for PS in (64, 128, 256, 512, 1024, 2048, 4096):
            if PS > 4 * (L + 8) + 64:
                continue
            ws1 = ops.decode_workspace(1, Hq, Hkv, D, L + 8, dev, PS=PS)
            t = timeit(lambda: ops.decode_step_attention(q1, kc1, vc1, slot, slot + 1, Hq, slot, cos, sin, workspace=ws1,
                                                         out=o1))
            r = dict(kind="attn_decode_fused_ps", B=1, L=L, PS=PS, NP=(L + 8 + PS - 1) // PS, us=t)
            res.append(r)
            print(json.dumps(r), flush=True)
    # one decode layer: fused (norm folded, residual epilogues, SwiGLU epilogue) vs unfused
    for M in ((1, 16, 32, 64) if want("layer") else ()):
        Hs, Fs = H, F
        x = torch.randn(M, Hs, device=dev, dtype=torch.bfloat16)
        resid = torch.randn_like(x)
        lnw = torch.ones(Hs, device=dev, dtype=torch.bfloat16)
        wqkv = torch.randn(NQKV, Hs, device=dev, dtype=torch.bfloat16) / 64
        wo = torch.randn(Hs, Hs, device=dev, dtype=torch.bfloat16) / 64
        wgu = torch.randn(2 * Fs, Hs, device=dev, dtype=torch.bfloat16) / 64
        wd = torch.randn(Hs, Fs, device=dev, dtype=torch.bfloat16) / 128
        att = torch.randn(M, Hs, device=dev, dtype=torch.bfloat16)

        def fused():
            q = ops.gemm_decode(x, wqkv, norm_eps=1e-5)
            h = ops.gemm_decode(att, wo, residual=x)
            f = ops.gemm_decode(h, wgu, act=ops.ACT_SWIGLU, norm_eps=1e-5)
            return ops.gemm_decode(f, wd, residual=h), q

        def unfused():
            y, h0 = ops.rms_norm(x, lnw, 1e-5, resid)
            q = ops.gemm(y, wqkv)
            a = ops.gemm(att, wo)
            y2, h = ops.rms_norm(a, lnw, 1e-5, h0)
            gu = ops.gemm(y2, wgu)
            return ops.gemm(ops.swiglu(gu), wd), q

        pass  # single (hand-written) GEMM path since round 2
        tu = timeit(unfused)
        tf = timeit(fused)
        pass  # single (hand-written) GEMM path since round 2
        r = dict(kind="decode_layer", M=M, fused_us=tf, unfused_us=tu)
        res.append(r)
        print(json.dumps(r), flush=True)
    # split-K sweep of the M <= 64 ring kernel (cold weights)
    for M in ((64,) if want("m64sweep") else ()):
        for name, N, K in gemms:
            ncopy = max(2, int(1.2e9 // (N * K * 2)))
            ws_ = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) / math.sqrt(K) for _ in range(ncopy)]
            a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            it = [0]

            def run_m64():
                it[0] = (it[0] + 1) % ncopy
                return ops.gemm(a, ws_[it[0]])

            for sp in (0, 1, 2, 4, 8, 16):
                if (K // 64) // max(sp, 1) < 2:
                    continue
                C.set_tuning({"m64_split": sp})
                t = timeit(run_m64, iters=ncopy * 2)
                r = dict(kind="m64_split", name=name, M=M, split=sp, us=t, gbs=2 * N * K / t / 1e3)
                res.append(r)
                print(json.dumps(r), flush=True)
            C.set_tuning({"m64_split": 0})
            del ws_
        torch.cuda.empty_cache()
    # LoRA-fused vs separate
    for M in ((2048, 8192) if want("lora") else ()):
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
    for B, S in (((16, 384), (4, 2048)) if want("attn") else ()):
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
    for B, L in (((1, 512), (64, 512), (64, 2048)) if want("decode") else ()):
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
        # fused rope + append + attention + combine (Smax > L as in generation)
        kc2 = torch.randn(B, Hkv, L + 64, D, device=dev, dtype=torch.bfloat16)
        vc2 = torch.randn_like(kc2)
        slot = torch.full((B,), L - 1, device=dev, dtype=torch.int32)
        alen = slot + 1
        cos, sin = ops.reference.rope_tables(D, 8192, 10000.0, dev)
        ws2 = ops.decode_workspace(B, Hq, Hkv, D, L + 64, dev)
        t2 = timeit(lambda: ops.decode_step_attention(q, kc2, vc2, slot, alen, Hq, slot, cos, sin, workspace=ws2,
                                                      out=out))
        t_rope = timeit(lambda: ops.rope_qkv_(q, slot, cos, sin, Hq, Hkv, D, S=1, k_cache=kc2, v_cache=vc2,
                                              slot_base=slot))
        r = dict(kind="attn_decode_fused", B=B, L=L, us=t2, unfused_us=t + t_rope, gbs=byts / t2 / 1e3)
        res.append(r)
        print(json.dumps(r), flush=True)
    # norm / logprob / sampler
    if not want("misc"):
        if args.json:
            with open(args.json, "w") as f:
                json.dump(res, f, indent=1)
        return
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
    for B_, k_, p_ in ((64, 50, 0.9), (1, 50, 0.9), (1, 50, 1.0), (64, 50, 1.0), (1, 0, 1.0), (64, 0, 1.0)):
        t = timeit(lambda: ops.sample(lg[:B_], 1 / 0.7, top_k=k_, top_p=p_, seed=1, offset=off))
        r = dict(kind="sample", B=B_, top_k=k_, top_p=p_, us=t)
        res.append(r)
        print(json.dumps(r), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
