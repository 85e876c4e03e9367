"""fp8 (e4m3fn) inference path: quantisation, W8A8 / W8A16 GEMM semantics, model integration (CPU
reference implementations; the HIP kernels are checked against these in test_kernels_gpu.py)."""
import torch

from rag_tl_domainllm_optimizer_amd import models, ops
from rag_tl_domainllm_optimizer_amd.models.config import PRESETS


def test_quantize_roundtrip():
    torch.manual_seed(0)
    x = torch.randn(33, 256) * torch.logspace(-2, 2, 33)[:, None]
    q, s = ops.quantize_fp8(x.to(torch.bfloat16))
    assert q.dtype == torch.uint8 and s.shape == (33,)
    xr = ops.dequantize_fp8(q, s)
    rel = ((xr - x).abs() / x.abs().amax(1, keepdim=True)).max()
    assert rel < 1 / 16  # e4m3: 3 mantissa bits
    # the row max maps to 448 exactly
    assert torch.allclose(q.view(torch.float8_e4m3fn).float().abs().amax(1), torch.full((33,), 448.0))


def test_gemm_fp8_reference_forms():
    torch.manual_seed(1)
    w = torch.randn(64, 256) / 16
    wq, sw = ops.quantize_fp8(w.to(torch.bfloat16))
    for M in (3, 80):  # W8A16 and W8A8
        x = torch.randn(M, 256).to(torch.bfloat16)
        y = ops.gemm_fp8(x, wq, sw)
        yr = x.float() @ w.t()
        assert (y.float() - yr).abs().max() < 0.08 * yr.abs().max()


def test_model_fp8_logits_close():
    cfg = PRESETS["tiny-llama"]
    m = models.CausalLM(cfg, dtype=torch.float32, seed=3)
    m.add_lora(r=4)
    ids = torch.randint(5, cfg.vocab_size, (2, 20))
    with torch.no_grad():
        ref = m(ids)
        m.set_fp8(True)
        got = m(ids)
        m.set_fp8(False)
    err = (got - ref).abs().max() / ref.abs().max()
    assert err < 0.1, err
