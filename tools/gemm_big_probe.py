"""Hand-written token-parallel GEMMs (gemm_big) on the PPO / prefill shapes of Mistral-7B, against
hipBLASLt (torch.matmul, comparator only), one process, interleaved rounds, random operands.

    python tools/gemm_big_probe.py [--M 9632 44288] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def tuned(fn, **kw):
    def run():
        with ops.tuning(**kw):
            return fn()
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[9632])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--cases", default="", help="comma-separated subset of the case names")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--sweep", default="", help="tuning knob sweep, e.g. gemm_group_m=2,8,16: adds nt/nn cases "
                    "per value (nt@gemm_group_m=8, ...)")
    a = ap.parse_args()
    dev = "cuda"
    C = ops.native()
    H, F, NQKV, R = 4096, 14336, 6144, 64
    shapes = {"qkv": (NQKV, H), "o": (H, H), "gate_up": (2 * F, H), "down": (H, F)}
    for M in a.M:
        for name in a.shapes.split(","):
            N, K = shapes[name]
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / 64).to(torch.bfloat16)
            u = (torch.rand(M, R, device=dev) * 2 - 1).to(torch.bfloat16)
            ub = ((torch.rand(N, R, device=dev) * 2 - 1) / 64).to(torch.bfloat16)
            dy = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
            du = (torch.rand(M, R, device=dev) * 2 - 1).to(torch.bfloat16)
            ap_ = ((torch.rand(R, K, device=dev) * 2 - 1) / 64).to(torch.bfloat16)
            xp = torch.empty(M, K + 64, device=dev, dtype=torch.bfloat16)[:, :K]
            xp.copy_(x)
            wp = torch.empty(N, K + 64, device=dev, dtype=torch.bfloat16)[:, :K]
            wp.copy_(w)
            cases = {
                "nt_padx": lambda: ops.gemm_big(xp, w, 0, 0),
                "nt_padw": lambda: ops.gemm_big(x, wp, 0, 0),
                "nt_padxw": lambda: ops.gemm_big(xp, wp, 0, 0),
                "nt": lambda: ops.gemm_big(x, w, 0, 0),
                "nt_k64": lambda: ops.gemm_big(x[:, :64], w[:, :64], 0, 0),
                "lib_k64": lambda: torch.matmul(x[:, :64], w[:, :64].t()),
                "nt_lora": lambda: ops.gemm_big(x, w, 0, 0, u, ub),
                "lib_nt": lambda: torch.matmul(x, w.t()),
                "nt256": lambda: ops.gemm_big(x, w, 0, 0, bn=256),
                "nt128": lambda: ops.gemm_big(x, w, 0, 0, bn=128),
                "nn256": lambda: ops.gemm_big(dy, w, 0, 1, bn=256),
                "nn128": lambda: ops.gemm_big(dy, w, 0, 1, bn=128),
                "nn_lora256": lambda: ops.gemm_big(dy, w, 0, 1, du, ap_, bn=256),
                "nn": lambda: ops.gemm_big(dy, w, 0, 1),
                "nn_lora": lambda: ops.gemm_big(dy, w, 0, 1, du, ap_),
                "lib_nn": lambda: torch.matmul(dy, w),
            }
            if name == "gate_up":
                cases["nt_swiglu"] = lambda: ops.gemm_big(x, w, 0, 0, act=5)
            if name == "gate_up":
                cases["nt128_swiglu"] = lambda: ops.gemm_big(x, w, 0, 0, act=5, bn=128)
            for sp in (1, 2, 4, 5, 8, 12, 16):
                cases[f"split{sp}"] = (lambda sp=sp: ops.gemm(x, w, nsplit=sp))
                if name == "gate_up":
                    cases[f"split{sp}_swiglu"] = (lambda sp=sp: ops.gemm(x, w, act=5, nsplit=sp))
            cases["auto"] = lambda: ops.gemm(x, w, act=5 if name == "gate_up" else 0)
            if a.cases:
                cases = {k: v for k, v in cases.items() if k in a.cases.split(",")}
            if a.sweep:
                knob, vals = a.sweep.split("=")
                for v in vals.split(","):
                    kw = {knob: float(v) if "." in v else int(v)}
                    cases[f"nt@{v}"] = tuned(lambda: ops.gemm_big(x, w, 0, 0), **kw)
                    cases[f"nn@{v}"] = tuned(lambda: ops.gemm_big(dy, w, 0, 1), **kw)
                    if name == "gate_up":
                        cases[f"sw@{v}"] = tuned(lambda: ops.gemm_big(x, w, 0, 0, act=5), **kw)
            res = {k: [] for k in cases}
            for _ in range(a.rounds):
                for k, fn in cases.items():
                    res[k].append(timeit(fn, a.iters))
            fl = 2 * M * N * K
            line = " ".join(f"{k}={statistics.median(v):7.1f}us({fl / statistics.median(v) / 1e6:5.0f}TF)"
                            for k, v in res.items())
            print(f"M={M} {name:8s} N={N} K={K}: {line}", flush=True)


if __name__ == "__main__":
    main()
