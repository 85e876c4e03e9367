"""Property-based (hypothesis) sweeps of the HIP kernels over ragged shapes against the fp32
PyTorch oracles in ops/reference.py (SURVEY §4.2 'op unit tests ... hypothesis for ragged sizes').
Example counts are kept small: every example is a few kernel launches on the GPU."""
import math

import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from rag_tl_domainllm_optimizer_amd import ops  # noqa: E402
from rag_tl_domainllm_optimizer_amd.ops import reference as ref  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
SET = settings(max_examples=12, deadline=None, derandomize=True)


def _close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * (b.abs().max().item() + 1e-6), err


@SET
@given(M=st.integers(1, 700), n8=st.integers(1, 150), k64=st.integers(1, 12), act=st.sampled_from([0, 1, 4]),
       lora=st.booleans(), seed=st.integers(0, 1 << 16))
def test_gemm_ragged(M, n8, k64, act, lora, seed):
    torch.manual_seed(seed)
    N, K = 8 * n8, 64 * k64
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / math.sqrt(K)
    u = torch.randn(M, 64, device=DEV, dtype=torch.bfloat16) if lora else None
    ub = torch.randn(N, 64, device=DEV, dtype=torch.bfloat16) * 0.1 if lora else None
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    _close(ops.gemm(a, w, u, ub, b, act), ref.gemm(a, w, u, ub, b, act, out_f32=True))


@SET
@given(T=st.integers(1, 300), h8=st.integers(1, 1024), res=st.booleans(), seed=st.integers(0, 1 << 16))
def test_rmsnorm_ragged(T, h8, res, seed):
    torch.manual_seed(seed)
    H = 8 * h8
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    r = torch.randn_like(x) if res else None
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    y, h = ops.rms_norm(x, w, 1e-5, r)
    yr, hr, _, _ = ref.norm(x, w, None, 1e-5, r)
    _close(y, yr)
    if res:
        assert torch.equal(h, hr)


@SET
@given(T=st.integers(1, 200), V=st.integers(2, 40000), temp=st.floats(0.5, 2.0), seed=st.integers(0, 1 << 16))
def test_logprob_ragged(T, V, temp, seed):
    torch.manual_seed(seed)
    logits = torch.randn(T, V, device=DEV, dtype=torch.bfloat16) * 3
    tgt = torch.randint(0, V, (T,), device=DEV)
    tgt[0] = -100
    lp, ent = ops.token_logprobs(logits, tgt, 1.0 / temp)
    lpr, entr, _, _ = ref.logprob(logits, tgt, 1.0 / temp)
    _close(lp, lpr, rtol=1e-3, atol=2e-3)
    _close(ent, entr, rtol=1e-3, atol=2e-3)


@SET
@given(B=st.integers(1, 3), S=st.integers(1, 300), D=st.sampled_from([64, 128]), G=st.sampled_from([1, 4]),
       causal=st.booleans(), seed=st.integers(0, 1 << 16))
def test_flash_attention_ragged(B, S, D, G, causal, seed):
    torch.manual_seed(seed)
    Hkv = 2
    Hq = Hkv * G
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    o = ops.flash_attention_qkv(qkv, B, S, Hq, Hkv, D, causal)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    _close(o, ref.attention(q, k, v, B, S, S, Hq, Hkv, D, causal)[0])
