"""Decode GEMMs at 16 < M <= 64 (small rollout batches): the M<=64 weight-streaming ring kernel
(ops.gemm default) vs the 256x128-tile split-K form of the token-parallel family.
    python tools/m64_probe.py [--M 32 64]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t(fn, iters=20):
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
    ap.add_argument("--M", type=int, nargs="+", default=[32, 64, 128])
    a = ap.parse_args()
    C = ops.native()
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for M in a.M:
        for name, (N, K) in shapes.items():
            x = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
            ws = [((torch.rand(N, K, device="cuda") - 0.5) / 64).to(torch.bfloat16) for _ in range(4)]  # > MALL
            act = 5 if name == "gate_up" else 0
            slabs = torch.empty(16 * M * N, device="cuda")
            cases = {"ring": lambda w: C.gemm(x, w, None, None, None, act, False, None)} if M <= 64 else {}
            for s in (1, 2, 4, 5, 8, 16):
                if act == 5 and s == 1:
                    cases["bn128_s1"] = lambda w: C.gemm_big(x, w, 0, 0, None, None, None, 5, 0, 1, None, None, None, 128)
                elif act == 0:
                    cases[f"bn128_s{s}"] = (lambda w, s=s: C.gemm_splitk(x, w, s, slabs, None, 0, None, None, 128))
                else:
                    cases[f"bn128_s{s}"] = (lambda w, s=s: C.gemm_splitk(x, w, s, slabs, None, 5, None, None, 128))
            res = {}
            for k, fn in cases.items():
                vals = []
                for r in range(3):
                    vals.append(t(lambda: [fn(w) for w in ws], 5) / len(ws))
                res[k] = statistics.median(vals)
            mb = N * K * 2 / 1e6
            print(f"M={M} {name:8s}: " + " ".join(f"{k}={v:6.1f}us({mb / v:4.1f}TB/s)" for k, v in res.items()),
                  flush=True)


if __name__ == "__main__":
    main()
