"""Token-parallel GEMM family (csrc/kernels/gemm_big.hip) against the fp32 PyTorch reference:
NT (forward), NN (dX, W read transposed in-kernel), TN (weight / LoRA gradients, split-K fp32
atomics), the LoRA K-extension, bias / activation epilogues, SwiGLU epilogue, ragged tails."""
import math

import pytest
import torch

from rag_tl_domainllm_optimizer_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, f"max err {err} (scale {scale})"


def _r(*shape, s=1.0):
    return (torch.randn(*shape, device=DEV) * s).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 200), (1024, 768, 1024), (77, 136, 4096),
                                   (513, 1024, 320), (2048, 2048, 2048)])
def test_nt(M, N, K):
    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW), a.float() @ w.float().t())


def test_nt_identity_asymmetric():
    n = 256
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(n * n, device=DEV).reshape(n, n) % 97).to(torch.bfloat16)
    torch.testing.assert_close(ops.gemm_big(a, w, ops.ROW, ops.ROW).float(), w.float().t())
    # NN: C = A W with W [K, N] read transposed
    torch.testing.assert_close(ops.gemm_big(a, w, ops.ROW, ops.KMAJ).float(), w.float())


@pytest.mark.parametrize("M,N,K", [(300, 512, 200), (1000, 4096, 1536), (64, 264, 128)])
def test_nn(M, N, K):
    dy, w = _r(M, K), _r(K, N, s=1 / math.sqrt(K))
    _close(ops.gemm_nn(dy, w), dy.float() @ w.float())


@pytest.mark.parametrize("T,P,Q,split", [(1000, 64, 512, 0), (4096, 512, 1024, 1), (776, 264, 136, 3)])
def test_tn_splitk(T, P, Q, split):
    T8 = T
    a, b = _r(T8, P), _r(T8, Q)
    got = ops.gemm_tn(a, b, nsplit=split)
    assert got.dtype == torch.float32
    _close(got, a.float().t() @ b.float(), rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("M", [200, 1100])
def test_lora_extension_nt_nn(M):
    K, N, R = 512, 768, 64
    x, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    u, ub = _r(M, R), _r(N, R, s=0.1)
    _close(ops.gemm_big(x, w, ops.ROW, ops.ROW, u, ub), x.float() @ w.float().t() + u.float() @ ub.float().t())
    # backward: dX = dY W + dU A_pad, A_pad [R, K] read transposed like W
    dy, du, ap = _r(M, N), _r(M, R), _r(R, K, s=0.1)
    _close(ops.gemm_nn(dy, w, du, ap), dy.float() @ w.float() + du.float() @ ap.float())


def test_bias_act_f32():
    M, N, K = 333, 384, 256
    a, w, b = _r(M, K), _r(N, K, s=1 / math.sqrt(K)), _r(N)
    for act in (0, 1, 2, 3, 4):
        want = ops.reference.apply_act(a.float() @ w.float().t() + b.float(), act)
        _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, bias=b, act=act), want)
    want = a.float() @ w.float().t() + b.float()
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, bias=b, out_mode=1), want, rtol=5e-3, atol=5e-3)


def test_swiglu_epilogue():
    M, F, K = 300, 512, 256
    x, w = _r(M, K), _r(2 * F, K, s=1 / math.sqrt(K))
    pre = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    f = ops.gemm_big(x, w, ops.ROW, ops.ROW, act=ops.ACT_SWIGLU, out2=pre)
    want_pre = (x.float() @ w.float().t()).to(torch.bfloat16)
    _close(pre, want_pre)
    want = torch.nn.functional.silu(want_pre[:, :F].float()) * want_pre[:, F:].float()
    _close(f, want)


def test_poisoned_output_fully_written():
    """Every output element is written (NaN-poisoned buffer, ragged M / N)."""
    M, N, K = 259, 264, 192
    a, w = _r(M, K), _r(N, K)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.gemm_big(a, w, ops.ROW, ops.ROW, out=out)
    assert torch.isfinite(out).all()


@pytest.mark.parametrize("M,N,K,split", [(256, 6144, 4096, 0), (200, 1024, 512, 3), (130, 768, 1024, 16)])
def test_splitk_small_m(M, N, K, split):
    x, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    want = x.float() @ w.float().t()
    _close(ops.gemm(x, w, nsplit=split), want)
    res = _r(M, N)
    _close(ops.gemm(x, w, residual=res, nsplit=split), want.to(torch.bfloat16).float() + res.float())
    f = ops.gemm(x, w, act=ops.ACT_SWIGLU, nsplit=split)
    pre = want.to(torch.bfloat16).float()
    F = N // 2
    _close(f, torch.nn.functional.silu(pre[:, :F]) * pre[:, F:])


@pytest.mark.parametrize("M,K,R", [(300, 4096, 64), (1000, 14336, 64), (77, 520, 128)])
def test_small_tile_narrow(M, K, R):
    """64x64-tile kernel: U = X A^T (ROW/ROW), dU = dY UB (ROW/KMAJ), bf16 out; TN split-K atomics."""
    x, a = _r(M, K), _r(R, K, s=1 / math.sqrt(K))
    _close(ops.native().gemm_small(x, a, ops.ROW, ops.ROW, 0, 1), x.float() @ a.float().t())
    ub = _r(K, R, s=1 / math.sqrt(K))
    _close(ops.native().gemm_small(x, ub, ops.ROW, ops.KMAJ, 0, 1), x.float() @ ub.float())
    t = _r(M, R)
    _close(ops.gemm_tn(t, x), t.float().t() @ x.float(), rtol=5e-3, atol=5e-3)
    _close(ops.gemm_tn(x, t), x.float().t() @ t.float(), rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("bm", [64, 128])
@pytest.mark.parametrize("M,K,R", [(300, 4096, 64), (1000, 1024, 64), (77, 520, 128), (200, 192, 64)])
def test_small_tile_bm(M, K, R, bm):
    """64x64 and 128x64 tiles of the narrow-product kernel, every layout it serves, bf16 / fp32 /
    split-K atomic outputs, partial tiles along M and K."""
    nat = ops.native()
    x, a = _r(M, K), _r(R, K, s=1 / math.sqrt(K))
    _close(nat.gemm_small(x, a, ops.ROW, ops.ROW, 0, 1, None, bm), x.float() @ a.float().t())
    ub = _r(K, R, s=1 / math.sqrt(K))
    _close(nat.gemm_small(x, ub, ops.ROW, ops.KMAJ, 0, 1, None, bm), x.float() @ ub.float())
    acc = torch.zeros(M, R, device=DEV)
    nat.gemm_small(x, ub, ops.ROW, ops.KMAJ, 2, 3, acc, bm)
    _close(acc, x.float() @ ub.float(), rtol=5e-3, atol=5e-3)
    t = _r(M, R)  # TN: [K, R] = x^T t and [R, K] = t^T x, token reduction split 4 ways
    out = torch.zeros(K, R, device=DEV)
    nat.gemm_small(x, t, ops.KMAJ, ops.KMAJ, 2, 4, out, bm)
    _close(out, x.float().t() @ t.float(), rtol=5e-3, atol=5e-3)
    out2 = torch.zeros(R, K, device=DEV)
    nat.gemm_small(t, x, ops.KMAJ, ops.KMAJ, 2, 4, out2, bm)
    _close(out2, t.float().t() @ x.float(), rtol=5e-3, atol=5e-3)
    o32 = nat.gemm_small(x, a, ops.ROW, ops.ROW, 1, 1, None, bm)
    _close(o32, x.float() @ a.float().t(), rtol=5e-3, atol=5e-3)


# ---- 256x128 tiles (decode at M <= 512, last partial wave of large GEMMs) and the wave planner ----
@pytest.mark.parametrize("bn", [128, 256, 0])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (300, 520, 200), (77, 136, 4096), (2900, 1024, 192)])
def test_bn_forms_nt_nn(bn, M, N, K):
    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    ref_nt = a.float() @ w.float().t()
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, bn=bn), ref_nt)
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, out_mode=1, bn=bn), ref_nt, rtol=5e-3, atol=5e-3)
    wk = _r(K, N, s=1 / math.sqrt(K))  # NN: C = A W, W [K, N]
    _close(ops.gemm_big(a, wk, ops.ROW, ops.KMAJ, bn=bn), a.float() @ wk.float())
    # residual epilogue, poisoned output fully written
    r = _r(M, N)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.gemm_big(a, w, ops.ROW, ops.ROW, out=out, residual=r, bn=bn)
    assert not torch.isnan(out).any()
    _close(out, ref_nt + r.float())


@pytest.mark.parametrize("bn", [128, 0])
def test_bn_lora_extension_and_swiglu(bn):
    M, K, F, R = 700, 512, 384, 64
    x, w = _r(M, K), _r(2 * F, K, s=1 / math.sqrt(K))
    u, ub = _r(M, R), _r(2 * F, R, s=0.1)
    _close(ops.gemm_big(x, w, ops.ROW, ops.ROW, u, ub, bn=bn), x.float() @ w.float().t() + u.float() @ ub.float().t())
    pre = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    y = ops.gemm_big(x, w, ops.ROW, ops.ROW, act=ops.ACT_SWIGLU, out2=pre, bn=bn)
    p_ref = (x.float() @ w.float().t()).to(torch.bfloat16)
    _close(pre, p_ref)
    g, up = p_ref[:, :F].float(), p_ref[:, F:].float()
    _close(y, torch.nn.functional.silu(g) * up)


@pytest.mark.parametrize("M,N,K,act", [(256, 6144, 4096, 0), (256, 28672, 512, 5), (256, 4096, 14336, 0),
                                       (200, 1000, 512, 0), (512, 32000, 256, 0)])
def test_decode_plan_m256(M, N, K, act):
    """ops.gemm at decode batch sizes (the 256x128 tile, split-K slabs or the SwiGLU epilogue)."""
    x, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    y = ops.gemm(x, w, act=act)
    ref_ = x.float() @ w.float().t()
    if act == ops.ACT_SWIGLU:
        ref_ = ref_.to(torch.bfloat16).float()
        ref_ = torch.nn.functional.silu(ref_[:, :N // 2]) * ref_[:, N // 2:]
    _close(y, ref_)
