"""Where does a batch-256 decode GEMM spend its time? Fixed (per-launch) cost vs per-K-step cost of
the 256x128-tile kernel: K sweep at 48 and 240 workgroups (bf16 out), split-K raw slabs (fp32 out,
no reduce), cold (4 weight copies > MALL share) and warm weights.
    python tools/m256_fixed_probe.py
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
    M = 256
    x = (torch.rand(M, 14336, device="cuda") - 0.5).to(torch.bfloat16)
    for N in (6144, 30720):
        for K in (256, 512, 1024, 2048, 4096):
            ws = [((torch.rand(N, K, device="cuda") - 0.5) / 64).to(torch.bfloat16) for _ in range(4)]
            xa = x[:, :K]
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            outf = torch.empty(M, N, device="cuda")
            cold = t(lambda: [C.gemm_big(xa, w, 0, 0, None, None, None, 0, 0, 1, out, None, None, 128) for w in ws]) / 4
            warm = t(lambda: [C.gemm_big(xa, ws[0], 0, 0, None, None, None, 0, 0, 1, out, None, None, 128)
                              for _ in ws]) / 4
            f32 = t(lambda: [C.gemm_big(xa, w, 0, 0, None, None, None, 0, 1, 1, outf, None, None, 128) for w in ws]) / 4
            fl = 2 * M * N * K
            print(f"N={N:6d} K={K:5d} wgs={N // 128:4d} steps={K // 64:3d}: bf16 cold {cold:7.1f}us warm {warm:7.1f}us "
                  f"f32 cold {f32:7.1f}us  ({fl / cold / 1e6:6.0f} TF/s cold, {N * K * 2 / cold / 1e6:4.1f} TB/s)",
                  flush=True)
            del ws
    for N, K in ((6144, 4096), (4096, 4096), (4096, 14336)):
        ws = [((torch.rand(N, K, device="cuda") - 0.5) / 64).to(torch.bfloat16) for _ in range(4)]
        xa = x[:, :K].contiguous()
        slabs = torch.empty(16 * M * N, device="cuda")
        res = []
        for s in (1, 2, 4, 5, 8, 12):
            v = t(lambda: [C.gemm_splitk_raw(xa, w, s, slabs, 128) for w in ws]) / 4
            res.append(f"s{s}={v:6.1f}us")
        print(f"raw split N={N} K={K}: " + " ".join(res), flush=True)
        del ws


if __name__ == "__main__":
    main()
