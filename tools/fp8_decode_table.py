"""Per-shape table: W8A16 fp8 decode GEMMs vs the bf16 decode GEMMs at M = 1 .. 64 (config 5).

Each projection of a decode layer (qkv, o, gate_up + SwiGLU, down) of Mistral-7B and Llama-2-13B
runs from cold weights (rotating copies larger than the 256 MB Infinity Cache, as in a decode step
that streams the whole model): bf16 = the kernel the bf16 decode step uses (M <= 16: tile-ordered
no-split GEMV; M > 16: the LDS-DMA ring), fp8 = ``ops.gemm_decode(fp8=Fp8Cache)`` (M <= 16:
tile-ordered fp8 GEMV; M > 16: the fp8 ring). One JSON line per case plus a summary table.

Usage: python tools/fp8_decode_table.py [--models mistral-7b,llama2-13b] [--ms 1,4,16,32,64]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402

SHAPES = {
    "mistral-7b": [("qkv", 6144, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, 5), ("down", 4096, 14336, 0)],
    "llama2-13b": [("qkv", 15360, 5120, 0), ("o", 5120, 5120, 0), ("gate_up", 27648, 5120, 5), ("down", 5120, 13824, 0)],
}


def timeit(fn, iters, warmup=4):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="mistral-7b,llama2-13b")
    ap.add_argument("--ms", default="1,2,4,8,16,24,32,48,64")
    ap.add_argument("--budget-gb", type=float, default=1.2)
    ap.add_argument("--splits", default="", help="also sweep the wide fp8 kernel's split-K at M > 16 (e.g. 1,2,4,8)")
    args = ap.parse_args()
    C = ops.native()
    dev = "cuda"
    rows = []
    for model in args.models.split(","):
        for name, N, K, act in SHAPES[model]:
            ncopy = max(2, int(args.budget_gb * 1e9 // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) / math.sqrt(K)).to(torch.bfloat16) for _ in range(ncopy)]
            shufs = [ops.ShufCache() for _ in ws]
            f8s = [ops.Fp8Cache() for _ in ws]
            for w, c in zip(ws, f8s):
                c.shuf(w)
            for M in [int(m) for m in args.ms.split(",")]:
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                it = [0]

                def bf16():
                    it[0] = (it[0] + 1) % ncopy
                    i = it[0]
                    return ops.gemm_decode(x, ws[i], act=act, shuf=shufs[i] if M <= 16 else None)

                def fp8():
                    it[0] = (it[0] + 1) % ncopy
                    i = it[0]
                    return ops.gemm_decode(x, ws[i], act=act, fp8=f8s[i])

                with torch.no_grad():
                    tb = timeit(bf16, ncopy * 4)
                    t8 = timeit(fp8, ncopy * 4)
                r = {"kind": "fp8_decode", "model": model, "name": name, "M": M, "N": N, "K": K,
                     "bf16_us": round(tb, 2), "fp8_us": round(t8, 2), "speedup": round(tb / t8, 3),
                     "bf16_gbs": round(2 * N * K / tb / 1e3, 1), "fp8_gbs": round(N * K / t8 / 1e3, 1)}
                if M > 16 and args.splits:
                    sw = {}
                    for sp in [int(v) for v in args.splits.split(",")]:
                        C.set_tuning({"wide_split": sp})
                        with torch.no_grad():
                            sw[sp] = round(timeit(fp8, ncopy * 4), 2)
                    C.set_tuning({"wide_split": 0})
                    r["fp8_split_us"] = sw
                rows.append(r)
                print(json.dumps(r), flush=True)
            del ws, shufs, f8s
            torch.cuda.empty_cache()
    print("\n| model | proj | " + " | ".join(f"M={m}" for m in args.ms.split(",")) + " |")
    print("|---|---|" + "---|" * len(args.ms.split(",")))
    for model in args.models.split(","):
        for name, *_ in SHAPES[model]:
            cells = [f"{r['bf16_us']:.1f} / {r['fp8_us']:.1f}" for r in rows if r["model"] == model and r["name"] == name]
            print(f"| {model} | {name} | " + " | ".join(cells) + " |")
    print("(cells: bf16 us / fp8 us, cold weights)")
    slower = [r for r in rows if r["speedup"] < 1.0]
    print(json.dumps({"fp8_slower_cases": [(r["model"], r["name"], r["M"], r["speedup"]) for r in slower]}))


if __name__ == "__main__":
    main()
