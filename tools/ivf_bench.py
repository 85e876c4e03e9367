"""IVF build/search timings on device: train (k-means on a 65k sample),
add 100k vectors (one shot and in 10 increments), search 256 queries, recall@10 vs flat.

    python tools/ivf_bench.py [--n 100000] [--d 384] [--nlist 512] [--nprobe 16] [--metric ip]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rag_tl_domainllm_optimizer_amd.retrieval import FlatIndex, IVFIndex  # noqa: E402


def clock(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--d", type=int, default=384)
    ap.add_argument("--nlist", type=int, default=512)
    ap.add_argument("--nprobe", type=int, default=16)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--niter", type=int, default=20)
    ap.add_argument("--metric", default="ip")
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    cen = torch.nn.functional.normalize(torch.randn(2048, a.d, device=dev, generator=g), dim=-1)
    x = cen[torch.randint(0, 2048, (a.n,), device=dev, generator=g)] + 0.03 * torch.randn(a.n, a.d, device=dev,
                                                                                         generator=g)
    x = torch.nn.functional.normalize(x, dim=-1)
    q = torch.nn.functional.normalize(x[:a.nq] + 0.02 * torch.randn(a.nq, a.d, device=dev, generator=g), dim=-1)
    res = {"n": a.n, "d": a.d, "nlist": a.nlist, "nprobe": a.nprobe, "nq": a.nq, "metric": a.metric}
    for rep in range(2):  # first pass warms kernels / allocator
        ivf = IVFIndex(a.d, a.nlist, a.metric, dev, a.nprobe)
        _, res["train_ms"] = clock(lambda: ivf.train(x, niter=a.niter))
        _, res["add_ms"] = clock(lambda: ivf.add(x))
        inc = IVFIndex(a.d, a.nlist, a.metric, dev, a.nprobe)
        inc.train(x, niter=a.niter)
        step = a.n // 10
        _, res["add_10x_ms"] = clock(lambda: [inc.add(x[s:s + step]) for s in range(0, a.n, step)])
        (_, ii), res["search_ms"] = clock(lambda: ivf.search(q, 10))
        flat = FlatIndex(a.d, a.metric, dev)
        flat.add(x)
        (_, fi), res["flat_search_ms"] = clock(lambda: flat.search(q, 10))
    res["recall@10"] = sum(len(set(u.tolist()) & set(v.tolist())) for u, v in zip(fi, ii)) / fi.numel()
    res["maxlen"] = ivf.maxlen
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
