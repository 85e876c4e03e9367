"""Batch-256 decode GEMMs: the production forms (256x128 tiles; qkv / o / down split-K into fp32
slabs, gate_up unsplit with the SwiGLU epilogue) vs 256x256 tiles streamed over every CU (stream-K
with no data-parallel part, bf16 out: tuning gemm_streamk = 2, bn 0). Back-to-back launches over 4
weight copies (cold weights, as in a decode step), results checked against fp32. Measured with
streamk_plan accepting fewer tiles than CUs (full == 0), reverted after this measurement
(profiles/r4/m256_all_streamk_vs_split.log: 2.3-2.7x slower).

    python tools/r4/m256_streamk_probe.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import splitk_plan  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    vals = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        vals.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(vals)


def main():
    C = ops.native()
    M = 256
    shapes = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "down": (4096, 14336, 0), "gate_up": (28672, 4096, 1)}
    for name, (N, K, swiglu) in shapes.items():
        act = ops.ACT_SWIGLU if swiglu else 0
        x = ((torch.rand(M, K, device="cuda") * 2 - 1)).to(torch.bfloat16)
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) / 64).to(torch.bfloat16) for _ in range(4)]
        ref = x.float() @ ws[0].float().t()
        if swiglu:
            F = N // 2
            ref = torch.nn.functional.silu(ref[:, :F].bfloat16().float()) * ref[:, F:].bfloat16().float()
        s, _ = splitk_plan(M, N, K, act)
        nout = N // 2 if swiglu else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        if s > 1:
            slabs = torch.empty(s * M * N, device="cuda")
            prod = timed(lambda: [C.gemm_splitk_raw(x, w, s, slabs, 128) for w in ws]) / 4
            C.gemm_splitk_raw(x, ws[0], s, slabs, 128)
            got_p = slabs[:s * M * N].view(s, M, N).sum(0)
            pname = f"256x128 split {s} -> fp32 slabs (+{s * M * N * 4 / 1e6:.0f} MB for the consumer)"
        else:
            prod = timed(lambda: [ops.gemm_big(x, w, ops.ROW, ops.ROW, act=act, out=out, bn=128) for w in ws]) / 4
            got_p = ops.gemm_big(x, ws[0], ops.ROW, ops.ROW, act=act, bn=128).float()
            pname = "256x128 unsplit"
        with ops.tuning(gemm_streamk=2):
            sk = timed(lambda: [ops.gemm_big(x, w, ops.ROW, ops.ROW, act=act, out=out, bn=0) for w in ws]) / 4
            got_s = ops.gemm_big(x, ws[0], ops.ROW, ops.ROW, act=act, bn=0).float()
            dirty = C.streamk_dirty_tickets()
        e_p = float((got_p - ref).abs().max() / ref.abs().max())
        e_s = float((got_s - ref).abs().max() / ref.abs().max())
        print(f"M=256 {name:7s} N={N:5d} K={K:5d} w={N * K * 2 / 1e6:4.0f}MB: {pname}: {prod:6.1f} us (err {e_p:.1e}) | "
              f"256x256 all-stream-K bf16: {sk:6.1f} us (err {e_s:.1e}, dirty tickets {dirty})", flush=True)
        del ws


if __name__ == "__main__":
    main()
