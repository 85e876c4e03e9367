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


# ---- 4-wave tiles (bn 3: 192 x 256, 96 x 128 per wave; bn 4: 256 x 256, 128 x 128 per wave) ----
@pytest.mark.parametrize("bn", [3, 4])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 224), (77, 136, 4096), (1000, 768, 1024),
                                   (2900, 1024, 192), (193, 6144, 4096)])
def test_w4_nt(bn, M, N, K):
    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    ref_nt = a.float() @ w.float().t()
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, bn=bn), ref_nt)
    _close(ops.gemm_big(a, w, ops.ROW, ops.ROW, out_mode=1, bn=bn), ref_nt, rtol=5e-3, atol=5e-3)
    r = _r(M, N)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.gemm_big(a, w, ops.ROW, ops.ROW, out=out, residual=r, bn=bn)
    assert not torch.isnan(out).any()
    _close(out, ref_nt + r.float())


@pytest.mark.parametrize("bn", [3, 4])
def test_w4_identity_bias_act_lora_swiglu(bn):
    n = 512
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(n * n, device=DEV).reshape(n, n) % 97).to(torch.bfloat16)
    torch.testing.assert_close(ops.gemm_big(a, w, ops.ROW, ops.ROW, bn=bn).float(), w.float().t())
    M, K, F, R = 700, 512, 384, 16
    x, wg = _r(M, K), _r(2 * F, K, s=1 / math.sqrt(K))
    b = _r(2 * F)
    for act in (0, 1, 2, 3, 4):
        want = ops.reference.apply_act(x.float() @ wg.float().t() + b.float(), act)
        _close(ops.gemm_big(x, wg, ops.ROW, ops.ROW, bias=b, act=act, bn=bn), want)
    u, ub = _r(M, R), _r(2 * F, R, s=0.1)  # LoRA K-extension with a ragged (K2 = 16) step
    _close(ops.gemm_big(x, wg, ops.ROW, ops.ROW, u, ub, bn=bn), x.float() @ wg.float().t() + u.float() @ ub.float().t())
    pre = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
    y = ops.gemm_big(x, wg, ops.ROW, ops.ROW, u, ub, act=ops.ACT_SWIGLU, out2=pre, bn=bn)
    p_ref = (x.float() @ wg.float().t() + u.float() @ ub.float().t()).to(torch.bfloat16)
    _close(pre, p_ref)
    _close(y, torch.nn.functional.silu(p_ref[:, :F].float()) * p_ref[:, F:].float())


# ---- stream-K tail (gemm_big_kernel<..., SK = true>): the last partial wave of 256x256 tiles split
# over K across every CU, partial tiles handed to the last arriving unit ----
# (M, N, K): tiles = ceil(M/256) * N/256 > 256 CUs with a remainder; ragged M / K; 1-3 segments
_SK_SHAPES = [(4352, 4096, 1024), (4500, 4096, 1000), (2600, 6144, 2048), (9632, 6144, 4096)]


@pytest.mark.parametrize("M,N,K", _SK_SHAPES)
def test_streamk_nt_nn_matches_reference(M, N, K):
    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    r = _r(M, N)
    with ops.tuning(gemm_streamk=2):
        got = ops.gemm_big(a, w, ops.ROW, ops.ROW)
        out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        ops.gemm_big(a, w, ops.ROW, ops.ROW, out=out, residual=r)
        wk = _r(K, N, s=1 / math.sqrt(K))
        nn = ops.gemm_big(a, wk, ops.ROW, ops.KMAJ)
    want = a.float() @ w.float().t()
    _close(got, want)
    assert not torch.isnan(out).any()
    _close(out, want + r.float())
    _close(nn, a.float() @ wk.float())
    # the data-parallel planner on the same operands: same result up to the K-split summation order
    with ops.tuning(gemm_streamk=0):
        dp = ops.gemm_big(a, w, ops.ROW, ops.ROW)
    _close(got, dp, rtol=1e-2, atol=1e-2)
    torch.cuda.synchronize()
    assert ops.native().streamk_dirty_tickets() == 0


def test_streamk_lora_extension_and_swiglu():
    """The K-extension steps (LoRA) are part of the split K range; SwiGLU + pre-activation output
    from the reduced tile."""
    M, K, F, R = 4352, 1024, 2048, 64  # 17 x 16 = 272 tiles of the [gate; up] weight
    x, w = _r(M, K), _r(2 * F, K, s=1 / math.sqrt(K))
    u, ub = _r(M, R), _r(2 * F, R, s=0.1)
    with ops.tuning(gemm_streamk=2):
        y = ops.gemm_big(x, w, ops.ROW, ops.ROW, u, ub)
        pre = torch.empty(M, 2 * F, device=DEV, dtype=torch.bfloat16)
        f = ops.gemm_big(x, w, ops.ROW, ops.ROW, act=ops.ACT_SWIGLU, out2=pre)
        dy, du, ap = _r(M, 2 * F), _r(M, R), _r(R, K, s=0.1)
        dx = ops.gemm_nn(dy, w, du, ap)
    _close(y, x.float() @ w.float().t() + u.float() @ ub.float().t())
    p_ref = (x.float() @ w.float().t()).to(torch.bfloat16)
    _close(pre, p_ref)
    _close(f, torch.nn.functional.silu(p_ref[:, :F].float()) * p_ref[:, F:].float())
    _close(dx, dy.float() @ w.float() + du.float() @ ap.float())
    torch.cuda.synchronize()
    assert ops.native().streamk_dirty_tickets() == 0


def test_streamk_repeat_and_side_stream():
    """Tickets re-arm themselves: many launches back to back (and on a second stream with its own
    workspace) give identical results."""
    M, N, K = 4500, 4096, 1536
    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    with ops.tuning(gemm_streamk=2):
        first = ops.gemm_big(a, w, ops.ROW, ops.ROW)
        for _ in range(5):
            assert torch.equal(ops.gemm_big(a, w, ops.ROW, ops.ROW), first)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            side = ops.gemm_big(a, w, ops.ROW, ops.ROW)
        torch.cuda.current_stream().wait_stream(s)
        assert torch.equal(side, first)
    torch.cuda.synchronize()
    assert ops.native().streamk_dirty_tickets() == 0


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 200), (77, 136, 4096), (1000, 768, 1024),
                                   (2900, 1024, 192), (512, 512, 128), (768, 1024, 4160)])
def test_ring_nt_bitwise(M, N, K):
    """The 10-slot granule ring (tuning gemm_ring) runs the same MFMAs on the same operands in the same
    order as the two-buffer schedule: bitwise-equal outputs for 1-, 2- and many-step K, ragged K
    tails, partial row / column tiles, the LoRA K-extension, a residual, SwiGLU and RoPE epilogues."""
    from rag_tl_domainllm_optimizer_amd.ops import reference as ref

    a, w = _r(M, K), _r(N, K, s=1 / math.sqrt(K))
    u, ub = _r(M, 64), _r(N, 64, s=0.1)
    r = _r(M, N)
    outs = []
    for ring in (0, 1):
        with ops.tuning(gemm_ring=ring):
            y = ops.gemm_big(a, w, ops.ROW, ops.ROW, bn=256)
            yl = ops.gemm_big(a, w, ops.ROW, ops.ROW, u, ub, bn=0)
            yr = ops.gemm_big(a, w, ops.ROW, ops.ROW, residual=r, bn=256)
            outs.append((y, yl, yr))
    for x0, x1 in zip(*outs):
        assert torch.equal(x0, x1)
    _close(outs[1][0], a.float() @ w.float().t())
    if N % 512 == 0:
        res = []
        cos, sin = ref.rope_tables(128, 2048, 10000.0, DEV)
        pos = torch.randint(0, 2048, (M,), device=DEV, dtype=torch.int32)
        for ring in (0, 1):
            with ops.tuning(gemm_ring=ring):
                pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
                f = ops.gemm_big(a, w, ops.ROW, ops.ROW, act=ops.ACT_SWIGLU, out2=pre, bn=256)
                q = ops.native().gemm_rope(a, w, None, None, None, pos, cos, sin, N // 2, 128, bn=256)
                res.append((f, pre, q))
        for x0, x1 in zip(*res):
            assert torch.equal(x0, x1)


@pytest.mark.parametrize("M,N,K", [(300, 512, 200), (1000, 4096, 1536), (256, 256, 64), (777, 1024, 4160)])
def test_ring_nn_bitwise(M, N, K):
    """NN (dX = dY W) on the granule ring: bitwise the two-buffer schedule, with the LoRA
    K-extension and the SwiGLU-backward epilogue."""
    dy, w = _r(M, K), _r(K, N, s=1 / math.sqrt(K))
    du, ap = _r(M, 64), _r(64, N, s=0.1)
    pre = _r(M, 2 * N)
    outs = []
    for ring in (0, 1):
        with ops.tuning(gemm_ring=ring):
            a = ops.gemm_big(dy, w, ops.ROW, ops.KMAJ, bn=256)
            b = ops.gemm_big(dy, w, ops.ROW, ops.KMAJ, du, ap, bn=0)
            o = torch.empty(M, 2 * N, device=DEV, dtype=torch.bfloat16)
            c = ops.gemm_big(dy, w, ops.ROW, ops.KMAJ, du, ap, act=ops.ACT_DSWIGLU, out=o, residual=pre, bn=256)
            outs.append((a, b, c))
    for x0, x1 in zip(*outs):
        assert torch.equal(x0, x1)
    _close(outs[1][0], dy.float() @ w.float())
