#!/usr/bin/env python3
"""Run-to-run reproducibility of the LoRA backward TN products (dB_all = dY^T U at the update's
9632 tokens, N = 28672 gate_up and 6144 qkv; dA_all = dU^T X at K = 14336): the fp32-atomic split-K
form (ops.linear.gemm_tn) vs the fixed-order slab form (ops.linear._tn_slabs + a fixed-order sum),
10 repeats each on the same inputs: how many output elements differ from the first run, and time.
Usage (GPU box): python tools/r6/atomic_vs_slab_repro.py"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
L = importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear")


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    T = 9632
    cases = {"dB gate_up": (T, 28672, 64, True), "dB qkv": (T, 6144, 64, True), "dA down": (T, 64, 14336, False)}
    for name, (t, p, q, _) in cases.items():
        a = torch.randn(t, p, device=dev).to(torch.bfloat16)
        b = torch.randn(t, q, device=dev).to(torch.bfloat16)
        res = {}
        for form in ("atomic", "slab"):
            outs = []
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for i in range(10):
                if i == 1:
                    ev[0].record()
                if form == "atomic":
                    outs.append(L.gemm_tn(a, b).clone())
                else:
                    ws, ns = L._tn_slabs(a, b, ("probe", p, q))
                    outs.append(ws.view(ns, p, q).sum(0))
            ev[1].record()
            torch.cuda.synchronize()
            diff = max(int((o != outs[0]).sum()) for o in outs[1:])
            res[form] = (diff, ev[0].elapsed_time(ev[1]) / 9 * 1e3)
        print(f"{name:12s} [{p} x {q}] atomic: {res['atomic'][0]:9d} of {p * q} elements differ across 10 runs "
              f"({res['atomic'][1]:6.1f} us) | slabs: {res['slab'][0]} differ ({res['slab'][1]:6.1f} us incl. torch sum)",
              flush=True)


if __name__ == "__main__":
    main()
