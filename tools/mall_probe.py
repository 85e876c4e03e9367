import torch, sys, os, json
sys.path.insert(0, '/root/repo')
from rag_tl_domainllm_optimizer_amd import ops
dev = 'cuda'
pass  # single (hand-written) GEMM path since round 2
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
for name, N, K in [("o", 4096, 4096), ("qkv", 6144, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]:
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    out = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
    acc = torch.zeros(1, device=dev)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    res = {}
    for mode in ("cold", "warm"):
        ts = []
        for it in range(6):
            flush.add_(1.0)  # evict
            if mode == "warm":
                torch.sum(w.view(torch.int16), dtype=torch.int32)  # read all weights (default policy)
            torch.cuda.synchronize()
            e[0].record(); ops.gemm(x, w, out=out); e[1].record()
            torch.cuda.synchronize()
            ts.append(e[0].elapsed_time(e[1]) * 1e3)
        res[mode] = round(sorted(ts)[len(ts)//2], 2)
    print(json.dumps(dict(name=name, MB=N*K*2/1e6, **res)), flush=True)
