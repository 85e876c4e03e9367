"""Row-pitch (channel camping) probe for the M = 256 decode GEMM shapes: the same GEMM with a dense
row pitch (K elements = 8 KiB for K = 4096) vs a padded pitch (K + pad), for X and W.
    python tools/pitch_probe.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    vals = []
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        vals.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(vals)


def main():
    C = ops.native()
    for M in (256, 2048):
        for name, N, K in (("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)):
            res = []
            for xpad in (0, 64):
                for wpad in (0, 64):
                    xb = (torch.rand(M, K + xpad, device="cuda") - 0.5).to(torch.bfloat16)
                    x = xb[:, :K]
                    wbs = [((torch.rand(N, K + wpad, device="cuda") - 0.5) / 64).to(torch.bfloat16) for _ in range(3)]
                    ws = [w[:, :K] for w in wbs]
                    if M == 256:
                        s = {"qkv": 5, "o": 8, "down": 8, "gate_up": 1}[name]
                        act = 5 if name == "gate_up" else 0
                        if act:
                            fn = lambda w: C.gemm_big(x, w, 0, 0, None, None, None, 5, 0, 1, None, None, None, 128)
                        else:
                            slabs = torch.empty(s * M * N, device="cuda")
                            fn = lambda w: C.gemm_splitk_raw(x, w, s, slabs, 128)
                    else:
                        fn = lambda w: C.gemm_big(x, w, 0, 0, None, None, None, 0, 0, 1, None, None, None, 0)
                    v = t(lambda: [fn(w) for w in ws]) / len(ws)
                    res.append(f"xpad{xpad}/wpad{wpad}={v:7.1f}us")
                    del wbs, ws
            print(f"M={M} {name:8s}: " + " ".join(res), flush=True)


if __name__ == "__main__":
    main()
