"""Is the batch-256 decode GEMM bound by fetching its weights? Same launch with a real [N, K]
weight (every row streamed from HBM) vs a stride-0 view of one row (every weight read an L2 hit)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops.linear import ROW  # noqa: E402

M = 256
x = torch.randn(M, 4096, device="cuda", dtype=torch.bfloat16)
for name, N, K, act in (("gate_up", 28672, 4096, 5), ("qkv_unsplit", 6144, 4096, 0)):
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(10)]
    one = torch.randn(1, K, device="cuda", dtype=torch.bfloat16).expand(N, K)
    for label, pick in (("hbm", lambda i: ws[i % len(ws)]), ("l2", lambda i: one)):
        for i in range(3):
            ops.gemm_big(x, pick(i), ROW, ROW, act=act, bn=128)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            ops.gemm_big(x, pick(i), ROW, ROW, act=act, bn=128)
        e1.record()
        torch.cuda.synchronize()
        print(f"M=256 {name:12s} weights from {label}: {e0.elapsed_time(e1) / 40 * 1e3:7.1f} us", flush=True)
