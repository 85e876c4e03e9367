"""Error map of the 4-wave NT GEMM tiles (bn 3 / 4) against fp32, per 16 x 16 block, small shapes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from rag_tl_domainllm_optimizer_amd import ops

torch.manual_seed(0)
for bn in (3, 4):
    for K in (32, 64, 128, 256, 512):
        M, N = 256, 256
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        ref = a.float() @ w.float().t()
        got = ops.gemm_big(a, w, 0, 0, out_mode=1, bn=bn)
        torch.cuda.synchronize()
        err = (got - ref).abs()
        blk = err.reshape(M // 16, 16, N // 16, 16).amax(dim=(1, 3))
        bad = (blk > 1e-2).nonzero().tolist()
        print(f"bn={bn} K={K}: max err {err.max().item():.4f}, bad 16x16 blocks {len(bad)}/{blk.numel()}", flush=True)
        if bad:
            rows = sorted(set(b[0] for b in bad)); cols = sorted(set(b[1] for b in bad))
            print("   bad block rows", rows[:20], "cols", cols[:20], flush=True)
            # is got a permutation of ref? check k-slice structure
            for kk in range(0, K, 32):
                part = a[:, kk:kk + 32].float() @ w[:, kk:kk + 32].float().t()
                print(f"   corr(got - ref, -kslice{kk}) = {torch.nn.functional.cosine_similarity((got - ref).flatten(), -part.flatten(), dim=0).item():.3f}")
            if K == 32:
                # identity probe: A = I rows -> C row m = W[:, m] ... show which k-chunks land
                e = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
                e[torch.arange(M), torch.arange(M) % K] = 1
                g2 = ops.gemm_big(e, w, 0, 0, out_mode=1, bn=bn)
                r2 = e.float() @ w.float().t()
                print("   identity probe rows wrong:", ((g2 - r2).abs().amax(1) > 1e-3).nonzero().flatten()[:32].tolist())
