"""Does a batch-1 decode GEMV run faster when its weight image was read shortly before (so it can
come from the memory-side Infinity Cache instead of HBM)?

Per projection (Mistral-7B qkv / o / gate_up / down, tile-ordered images, M = 1) and per condition,
REPS launches of the real gemv16 kernel, each preceded by:
  cold  - a 1 GiB read (evicts the 256 MB cache)
  sum   - the 1 GiB read, then a plain-load read of the weight image (torch sum)
  nt    - the 1 GiB read, then the GEMV itself (non-temporal loads) as the prefetch
Run under `rocprofv3 --kernel-trace` and pass the trace to --parse: the GEMV kernel durations are
split back into (projection, condition) blocks by launch order.

    rocprofv3 --kernel-trace -d gpurun_out/mall -o run -- python tools/r4/mall_probe.py
    python tools/r4/mall_probe.py --parse gpurun_out/mall
"""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = (("qkv", 6144, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 0))
CONDS = ("cold", "sum", "nt")


def run(reps):
    import torch

    from rag_tl_domainllm_optimizer_amd import ops

    flush = torch.ones(1 << 29, dtype=torch.bfloat16, device="cuda")  # 1 GiB
    x = torch.randn(1, 14336, dtype=torch.bfloat16, device="cuda") * 0.1
    for name, N, K, act in SHAPES:
        w = torch.randn(N, K, dtype=torch.bfloat16, device="cuda") * 0.02
        sc = ops.ShufCache()
        wimg = sc.get(w)
        xa = x[:, :K].contiguous()
        a = ops.ACT_SWIGLU if act else 0
        for cond in CONDS:
            for _ in range(reps):
                flush.sum()
                if cond == "sum":
                    wimg.sum()
                elif cond == "nt":
                    ops.gemm_decode(xa, w, act=a, shuf=sc)
                ops.gemm_decode(xa, w, act=a, shuf=sc)
            torch.cuda.synchronize()
        print(name, "done", flush=True)
        del w, sc, wimg


def parse(d, reps):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    g = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "gemv16" in r["Kernel_Name"]]
    sums = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
            if "reduce" in r["Kernel_Name"].lower()]
    i = 0
    for name, N, K, _ in SHAPES:
        mb = N * K * 2 / 1e6
        for cond in CONDS:
            per = 2 if cond == "nt" else 1
            blk = g[i:i + reps * per]
            i += reps * per
            t = sorted(blk[per - 1::per])[reps // 2] / 1e3
            extra = ""
            if cond == "nt":
                p = sorted(blk[0::per])[reps // 2] / 1e3
                extra = f"  (prefetching GEMV itself {p:.1f} us)"
            print(f"{name:8s} {mb:6.1f} MB  {cond:4s}  median {t:6.1f} us  {mb / t:5.2f} TB/s{extra}")
    print(f"({len(g)} GEMV launches parsed, {len(sums)} reductions)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--parse", default="")
    a = ap.parse_args()
    if a.parse:
        parse(a.parse, a.reps)
    else:
        run(a.reps)


if __name__ == "__main__":
    main()
