"""The fused MLP autograd node (ops.swiglu_mlp: gate/up GEMM with the SwiGLU epilogue, down GEMM,
backward with the SwiGLU backward inside the down projection's dX GEMM) equals the two-linear form
in outputs and in every gradient (input, LoRA A / B of gate, up and down, full weights). CPU oracles."""
import pytest
import torch

from rag_tl_domainllm_optimizer_amd import ops


def _group(names, n_out, K, r, rows, seed):
    g = torch.Generator().manual_seed(seed)
    a = [torch.nn.Parameter(torch.randn(r, K, generator=g) * 0.05) for _ in names]
    b = [torch.nn.Parameter(torch.randn(n, r, generator=g) * 0.05) for n in rows]
    c0 = [0] + [sum(rows[:i + 1]) for i in range(len(rows) - 1)]
    return ops.LoRAGroup(list(names), a, b, c0, [2.0] * len(names), n_out)


@pytest.mark.parametrize("lora,full", [(True, False), (False, True)])
def test_fused_mlp_matches_two_linears(lora, full):
    torch.manual_seed(0)
    M, H, F = 37, 64, 256
    x = torch.randn(M, H, requires_grad=True)
    w_gu = (torch.randn(2 * F, H) * 0.1).requires_grad_(full)
    w_d = (torch.randn(H, F) * 0.1).requires_grad_(full)
    lg = _group(["gate_proj", "up_proj"], 2 * F, H, 4, [F, F], 1) if lora else None
    ld = _group(["down_proj"], H, F, 4, [H], 2) if lora else None
    for g in (lg, ld):
        if g is not None:
            g.refresh(dtype=torch.float32)
    params = [p for g in (lg, ld) if g is not None for p in g.a + g.b] + ([w_gu, w_d] if full else [])
    gy = torch.randn(M, H)

    def grads(y):
        tensors = [x] + params
        return torch.autograd.grad((y * gy).sum(), tensors)

    y1 = ops.swiglu_mlp(x, w_gu, w_d, lg, ld, cpu=True)
    assert y1 is not None
    g1 = grads(y1)
    f = ops.linear(x, w_gu, act="swiglu", lora=lg)
    y2 = ops.linear(f, w_d, lora=ld)
    g2 = grads(y2)
    torch.testing.assert_close(y1, y2, rtol=1e-5, atol=1e-6)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
    assert all(a.abs().sum() > 0 for a in g1)


def test_fused_mlp_declines_dropout_and_no_grad():
    M, H, F = 8, 64, 256
    x = torch.randn(M, H, requires_grad=True)
    w_gu, w_d = torch.randn(2 * F, H), torch.randn(H, F)
    lg = _group(["gate_proj", "up_proj"], 2 * F, H, 4, [F, F], 1)
    lg.dropout = 0.1
    assert ops.swiglu_mlp(x, w_gu, w_d, lg, None, cpu=True) is None
    with torch.no_grad():
        assert ops.swiglu_mlp(x, w_gu, w_d, None, None, cpu=True) is None
