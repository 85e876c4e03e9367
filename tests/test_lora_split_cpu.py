"""Split plans of the LoRA narrow products (ops.linear._narrow / gemm_tn) measured in round 5
(profiles/r5/lora_narrow_split_sweep.log): the forward U = X A^T splits 3 ways into fixed-order fp32 slabs (round 6: deterministic), the
token reduction of dA / dB splits 4 ways on 64 output tiles and 8 above. The plans are host code:
checked here by intercepting the native launch."""
import importlib

import torch

L = importlib.import_module("rag_tl_domainllm_optimizer_amd.ops.linear")  # the module (ops.linear is the function)


class _Native:
    def __init__(self):
        self.calls = []

    def gemm_small(self, a, b, la, lb, out_mode, ns, out, bm):
        self.calls.append((la, lb, out_mode, ns, bm))
        R = b.shape[0] if lb == L.ROW else b.shape[1]
        if out_mode == 3:
            return torch.zeros(ns * a.shape[0], R, dtype=torch.float32)
        return out if out is not None else torch.zeros(a.shape[0], R, dtype=a.dtype)

    def splitk_reduce(self, slabs, ns, M, N, out):
        return out


def _run(monkeypatch, fn):
    nat = _Native()
    monkeypatch.setattr(L, "native", lambda: nat)
    monkeypatch.setattr(L, "on_gpu", lambda t: True)
    fn()
    return nat.calls


def test_forward_u_splits_into_slabs(monkeypatch):
    """The forward adapter product U = X A_pad^T splits 3 ways into fp32 slabs (out mode 3) summed in a
    fixed order — never fp32 atomics, whose arrival-order sums would make the scoring forward
    non-reproducible and batch-variant (ops.batch_invariant, PPO ratio / reference KL exactness)."""
    for K in (4096, 14336):
        x = torch.zeros(9632, K, dtype=torch.bfloat16)
        a = torch.zeros(64, K, dtype=torch.bfloat16)
        calls = _run(monkeypatch, lambda: L._narrow(x, a, L.ROW))
        assert [(c[2], c[3]) for c in calls] == [(3, 3)], (K, calls)
    # tiny reductions are not split
    calls = _run(monkeypatch, lambda: L._narrow(torch.zeros(300, 256, dtype=torch.bfloat16),
                                                torch.zeros(64, 256, dtype=torch.bfloat16), L.ROW))
    assert [c[3] for c in calls] == [1]
    # the backward dU = dY UB (KMAJ adapter image [N, Rp]): slabs too, ~3 workgroups per CU
    calls = _run(monkeypatch, lambda: L._narrow(torch.zeros(9632, 28672, dtype=torch.bfloat16),
                                                torch.zeros(28672, 64, dtype=torch.bfloat16), L.KMAJ))
    assert calls == [(L.ROW, L.KMAJ, 3, 6, 128)], calls


def test_backward_tn_products_into_slabs(monkeypatch):
    """dA_all = dU^T X and dB_all = dY^T U of the LoRA backward: token-split fp32 slabs (out mode 3,
    KMAJ x KMAJ) in a cached workspace, gemm_tn's tiles; 8 splits on 64x64 tiles, 2 on the 128x64
    tiles of gate_up's dB (profiles/r6/lora_narrow_sweep.log)."""
    T = 9632
    du = torch.zeros(T, 64, dtype=torch.bfloat16)
    for a, b, ns, bm in ((du, torch.zeros(T, 4096, dtype=torch.bfloat16), 8, 64),
                         (torch.zeros(T, 28672, dtype=torch.bfloat16), du, 2, 128)):
        out = []
        calls = _run(monkeypatch, lambda: out.append(L._tn_slabs(a, b, ("t", a.shape[1], b.shape[1]))))
        assert calls == [(L.KMAJ, L.KMAJ, 3, ns, bm)], calls
        ws, n = out[0]
        assert n == ns and ws.shape == (ns * a.shape[1], b.shape[1])
    L._WS.clear()


def test_adapter_gradient_token_splits(monkeypatch):
    T = 9632
    du = torch.zeros(T, 64, dtype=torch.bfloat16)
    cases = [(lambda: L.gemm_tn(du, torch.zeros(T, 4096, dtype=torch.bfloat16)), 4),    # dA, 64 tiles
             (lambda: L.gemm_tn(du, torch.zeros(T, 14336, dtype=torch.bfloat16)), 8),   # dA, 224 tiles
             (lambda: L.gemm_tn(torch.zeros(T, 4096, dtype=torch.bfloat16), du), 4),    # dB, 64 tiles
             (lambda: L.gemm_tn(torch.zeros(T, 6144, dtype=torch.bfloat16), du), 8)]    # dB, 96 tiles
    for fn, ns in cases:
        calls = _run(monkeypatch, fn)
        assert [c[3] for c in calls] == [ns], calls


class _NativeGemm:
    def __init__(self):
        self.calls = []

    def gemm(self, x, w, *a):
        self.calls.append("skinny")
        return torch.zeros(x.shape[0], w.shape[0], dtype=x.dtype)

    def gemm_splitk(self, x, w, s, *a):
        self.calls.append(f"splitk{s}")
        return torch.zeros(x.shape[0], w.shape[0], dtype=x.dtype)

    def gemm_big(self, a, b, la, lb, a2, b2, bias, act, out_mode, nsplit, out, out2, residual, bn):
        self.calls.append(f"big{nsplit}")
        return torch.zeros(a.shape[0], b.shape[0], dtype=a.dtype)


def test_batch_invariant_dispatch(monkeypatch):
    """ops.batch_invariant(): every token-parallel GEMM takes the unsplit 256-row kernel whatever M
    is (the per-M plan picks skinny kernels at M <= 64 and split-K at M <= 512 otherwise), per
    thread, nesting."""
    import threading

    nat = _NativeGemm()
    monkeypatch.setattr(L, "native", lambda: nat)
    monkeypatch.setattr(L, "on_gpu", lambda t: True)
    w = torch.zeros(4096, 4096, dtype=torch.bfloat16)
    for M in (8, 48, 300, 2000):
        L.gemm(torch.zeros(M, 4096, dtype=torch.bfloat16), w)
    assert nat.calls[0] == "skinny" and nat.calls[2].startswith("splitk") and nat.calls[3] == "big1", nat.calls
    nat.calls.clear()
    with L.batch_invariant():
        with L.batch_invariant():
            L.gemm(torch.zeros(8, 4096, dtype=torch.bfloat16), w)
        for M in (48, 300, 2000):
            L.gemm(torch.zeros(M, 4096, dtype=torch.bfloat16), w)
        other = []
        th = threading.Thread(target=lambda: (L.gemm(torch.zeros(8, 4096, dtype=torch.bfloat16), w),
                                              other.append(nat.calls[-1])))
        th.start()
        th.join()
    assert nat.calls[:4] == ["big1"] * 4, nat.calls
    assert other == ["skinny"]  # another thread keeps its own (default) plans
    L.gemm(torch.zeros(8, 4096, dtype=torch.bfloat16), w)
    assert nat.calls[-1] == "skinny"
