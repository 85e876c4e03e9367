"""Host-side cost of library GEMM calls on ROCm (hipBLASLt vs rocBLAS backends of torch.mm).

For each PPO-update GEMM shape: host issue time per call (no sync, queue kept busy) and device
time per call, under torch.backends.cuda.preferred_blas_library 'cublaslt' (hipBLASLt) and
'cublas' (rocBLAS)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, M, N, K, a_T, b_T)  C[M,N] = A[M,K] @ B[K,N]
    ("u=x@A^T", 7168, 64, 4096, False, True),
    ("dx=dy@W(qkv)", 7168, 4096, 6144, False, False),
    ("dx=dy@W(down)", 7168, 14336, 4096, False, False),
    ("du=dy@ub", 7168, 64, 6144, False, False),
    ("gA=du^T@x", 64, 4096, 7168, True, False),
    ("gB=dy^T@u", 6144, 64, 7168, True, False),
    ("merge ub@A", 4096, 4096, 64, False, False),
]


def main():
    dev = "cuda"
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        for name, M, N, K, at, bt in SHAPES:
            a = torch.randn(K, M, device=dev, dtype=torch.bfloat16).t() if at else \
                torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            b = torch.randn(N, K, device=dev, dtype=torch.bfloat16).t() if bt else \
                torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                torch.mm(a, b)
            torch.cuda.synchronize()
            torch.cuda._sleep(int(5e8))
            n = 50
            t0 = time.perf_counter()
            for _ in range(n):
                torch.mm(a, b)
            host = (time.perf_counter() - t0) / n * 1e6
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                torch.mm(a, b)
            e1.record()
            torch.cuda.synchronize()
            dev_us = e0.elapsed_time(e1) / n * 1e3
            print(json.dumps(dict(lib=lib, name=name, M=M, N=N, K=K, host_us=round(host, 1), dev_us=round(dev_us, 1),
                                  tflops=round(2 * M * N * K / dev_us / 1e6, 1))), flush=True)


if __name__ == "__main__":
    main()
